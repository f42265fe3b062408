# Fused two-level zero-guess restriction (fea_mg_zero_restrict2): bitwise tests, the whole GPU suite of the
# solver, then the metric cycle's kernel times under a trace
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03q; mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_mg.py -m gpu -x -q --timeout 120 --timeout-method thread -k "zero_restrict2 or prolong2 or pairs_restrictions" > $T/pytest_zr2.log 2>&1 || { echo "zr2 tests failed"; tail -40 $T/pytest_zr2.log; exit 1; }
tail -2 $T/pytest_zr2.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_configs.py tests/test_gpu_mid.py tests/test_gpu_dd.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/p4097 -o run -- python3 bench.py --no-cpu-baseline > $T/b4097.json 2> $T/b4097.err || { tail $T/b4097.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $T/b20.json 2> $T/b20.err || { tail $T/b20.err; exit 1; }
python3 -c "
import json,csv,glob
for f in ('b4097','b20'):
    d=json.load(open('$T/'+f+'.json')); print(f, d['ms_per_step'], d['value'])
f=glob.glob('$T/p4097/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:9]: print(f\"{r['Name'][:70]:72s} {int(r['Calls']):7d} {float(r['AverageNs'])/1000:8.2f}\")
"
