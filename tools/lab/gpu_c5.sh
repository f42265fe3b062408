# C5 (256 x 1025^2 fp32) lab: kernel traces of library variants, then PMC traffic of the in-tree build
#   bash tools/lab/gpu_c5.sh TAG LIB1 LIB2 ...   ("-" = the in-tree library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
A="--n 1024 --batch 256 --dtype f32 --no-cpu-baseline"
i=0
for L in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $T/v$i -o run -- python3 tools/lab/with_lib.py $L bench.py $A --steps 30 --warmup 2 --kernel-reps 2 > $T/v$i.json 2> $T/v$i.err || { tail $T/v$i.err; exit 1; }
  python3 tools/trace_summary.py $T/v$i > $T/v$i.txt
  echo "== [$L] $(python3 -c "import json; print(json.load(open('$T/v$i.json'))['ms_per_step']*1e3)") us"; head -${NLINES:-8} $T/v$i.txt
done
if [ -n "$PMC" ]; then
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $T/pmc_$c -o run -- python3 tools/lab/with_lib.py - bench.py $A --steps 3 --warmup 1 --kernel-reps 1 > $T/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail $T/pmc_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $(ls $T/pmc_FETCH_SIZE/*counter_collection.csv) $(ls $T/pmc_WRITE_SIZE/*counter_collection.csv) $T/pmc_traffic.json $T/pmc_summary.txt profiles/c5_pmc > /dev/null && head -14 $T/pmc_summary.txt
fi
