# usage: bash tools/gpu_check.sh TAG [bench args...]  — GPU tests, smoke, bench, kernel trace
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
T=gpurun_out/$1; shift
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest_gpu.log; exit 1; }
tail -2 $T/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { cat $T/smoke.log; exit 1; }
tail -1 $T/smoke.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $T/bench.json 2> $T/bench.err || { tail $T/bench.err; exit 1; }
cat $T/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline "$@" > $T/trace_bench.json 2>$T/trace.err || { tail $T/trace.err; exit 1; }
python3 tools/trace_summary.py $T/trace > $T/trace_summary.txt && head -22 $T/trace_summary.txt
