# HJac two-level launches: parity tests, then the MG-HJac 4097^2 fp64 cycle against a baseline build (A B A B) and
# a kernel trace of the in-tree build.   bash tools/lab/gpu_hmid.sh TAG "pytest -k expr" [BASE.so]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T; BASE=${3:-tools/lab/lib_prev.so}
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_hnet.py -m gpu -x -q -k "$2" --timeout 300 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
for i in 1 2; do for L in $BASE -; do
  timeout -k 10 300 python3 tools/lab/with_lib.py $L bench.py --smoother hjac --steps 200 --warmup 5 --no-cpu-baseline --kernel-reps 3 > $T/b.json 2> $T/b.err || { tail $T/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$T/b.json')); print('$L', round(d['ms_per_step']*1e3,1), 'us')"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof -o run -- python3 bench.py --smoother hjac --steps 200 --warmup 5 --no-cpu-baseline --kernel-reps 3 > $T/bp.json 2> $T/bp.err || { tail $T/bp.err; exit 1; }
python3 tools/trace_summary.py $T/prof > $T/trace.txt 2>&1 && head -30 $T/trace.txt
