# PMC HBM traffic per kernel (FETCH_SIZE / WRITE_SIZE passes) for several library builds (GPU box):
#   bash tools/lab/gpu_pmc_libs.sh TAG LIB1 LIB2 ...   ("-" = the in-tree library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
i=0
for L in "$@"; do
  i=$((i+1))
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $T/v${i}_$c -o run -- python3 tools/lab/with_lib.py $L bench.py --steps 20 --warmup 3 --no-cpu-baseline --kernel-reps 5 $BENCH_ARGS > $T/v${i}_$c.log 2>&1 || { echo "pmc $c failed"; tail $T/v${i}_$c.log; exit 1; }
  done
  python3 tools/pmc_traffic.py $(ls $T/v${i}_FETCH_SIZE/*counter_collection.csv) $(ls $T/v${i}_WRITE_SIZE/*counter_collection.csv) $T/v$i.json $T/v$i.txt > /dev/null
  echo "== [$L]"; head -${NLINES:-8} $T/v$i.txt
done
