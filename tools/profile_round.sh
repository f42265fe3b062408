# Round profile: PMC traffic passes, then the bench line and its kernel trace (same command).
#   bash tools/profile_round.sh TAG   (from the repo root, on the GPU box)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
T=gpurun_out/$1
mkdir -p $T
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $T/pmc_$c -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --kernel-reps 5 > $T/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail $T/pmc_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $(ls $T/pmc_FETCH_SIZE/*counter_collection.csv) $(ls $T/pmc_WRITE_SIZE/*counter_collection.csv) $T/pmc_traffic.json $T/pmc_summary.txt profiles/$1_pmc > /dev/null && head -12 $T/pmc_summary.txt
export FEANET_PMC_TRAFFIC=$T/pmc_traffic.json
timeout -k 10 300 python3 bench.py > $T/bench.json 2> $T/bench.err || { tail $T/bench.err; exit 1; }
cat $T/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- python3 bench.py > $T/trace_bench.json 2> $T/trace.err || { tail $T/trace.err; exit 1; }
python3 tools/trace_summary.py $T/trace > $T/trace_summary.txt && head -16 $T/trace_summary.txt
