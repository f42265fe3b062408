set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_hnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
for i in 1 2; do for L in tools/lab/lib_prev.so -; do
  timeout -k 10 300 python3 tools/lab/with_lib.py $L bench.py --smoother hjac --steps 20 --warmup 2 --no-cpu-baseline --kernel-reps 3 > $T/b.json 2> $T/b.err || { tail $T/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$T/b.json')); print('$L', round(d['ms_per_step']*1e3,1), 'us')"
done; done
