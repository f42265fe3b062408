set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
T=gpurun_out/r02b
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest_gpu.log; exit 1; }
tail -2 $T/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $T/bench20.json 2> $T/bench20.err || { tail $T/bench20.err; exit 1; }
timeout -k 10 300 python -u bench.py > $T/bench.json 2> $T/bench.err || { tail $T/bench.err; exit 1; }
python3 -c "
import json
for f in ('bench20','bench'):
    d=json.load(open('$T/'+f+'.json')); print(f, d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('cpu_baseline'))
"
