set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/mid1; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_gpu_mid.py tests/test_gpu_mg.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
timeout -k 10 100 python tools/lab/mid_trace.py > $T/mid.txt 2>&1; cat $T/mid.txt
bash tools/lab/gpu_trace_ab.sh mid1ab
