# PMC traffic of the C4-size (8193^2 fp64) and C3 (2049^2 two-material) kernels
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03l; mkdir -p $T
for cfg in "c4one:--n 8192 --steps 10 --warmup 2 --kernel-reps 3" "c3:--n 2048 --problem interface --steps 20 --warmup 2 --kernel-reps 3"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $T/${name}_$c -o run -- python3 bench.py --no-cpu-baseline $args > $T/${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; tail $T/${name}_$c.log; exit 1; }
  done
  python3 tools/pmc_traffic.py $(ls $T/${name}_FETCH_SIZE/*counter_collection.csv) $(ls $T/${name}_WRITE_SIZE/*counter_collection.csv) $T/${name}_traffic.json $T/${name}_summary.txt profiles/r03l_pmc > /dev/null
  echo "== $name"; head -14 $T/${name}_summary.txt
done
