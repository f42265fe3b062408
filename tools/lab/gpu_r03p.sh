# Coarse tail: the 65^2 / 6-level V(1,1) path as its own kernel (no scratch spills): parity + kernel times
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03p; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/p4097 -o run -- python3 bench.py --no-cpu-baseline > $T/b4097.json 2> $T/b4097.err || { tail $T/b4097.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/pc3 -o run -- python3 bench.py --no-cpu-baseline --n 2048 --problem interface --steps 200 > $T/bc3.json 2> $T/bc3.err || { tail $T/bc3.err; exit 1; }
python3 -c "
import json
for f in ('b4097','bc3'):
    d=json.load(open('$T/'+f+'.json')); print(f, d['ms_per_step'], d['value'])
"
for d in p4097 pc3; do f=$(ls $T/$d/*/run_kernel_stats.csv 2>/dev/null || ls $T/$d/run_kernel_stats.csv); echo "== $d"; head -12 $f | cut -d, -f1-4 | cut -c1-150; done
