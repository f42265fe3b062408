# parity of the HJac two-level launches, their phase trace, then the MG-HJac cycle A/B against tools/lab/lib_prev.so
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_hnet.py -m gpu -x -q -k "${2:-hmid or hjac}" --timeout 300 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
timeout -k 10 300 python3 tools/lab/hmid_trace.py > $T/trace.txt 2>&1 || { tail -20 $T/trace.txt; exit 1; }
grep hmid $T/trace.txt
for i in 1 2; do for L in tools/lab/lib_prev.so -; do
  timeout -k 10 300 python3 tools/lab/with_lib.py $L bench.py --smoother hjac --steps 200 --warmup 5 --no-cpu-baseline --kernel-reps 3 > $T/b.json 2> $T/b.err || { tail $T/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$T/b.json')); print('$L', round(d['ms_per_step']*1e3,1), 'us')"
done; done
