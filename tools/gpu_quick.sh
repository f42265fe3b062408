# usage: bash tools/gpu_quick.sh TAG [pytest selection...] — GPU tests (selection or all), then a short bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
T=gpurun_out/$1; shift
mkdir -p $T
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $T/pytest_gpu.log; exit 1; }
tail -3 $T/pytest_gpu.log
grep -h "solve .* cycles" $T/pytest_gpu.log || true
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $T/bench20.json 2> $T/bench20.err || { tail $T/bench20.err; exit 1; }
python3 -c "
import json
d=json.load(open('$T/bench20.json')); print('bench20', d['ms_per_step'], d['value'], d['roofline']['frac'])
"
