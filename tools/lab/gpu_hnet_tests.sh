set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_hnet.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest.log 2>&1 || { tail -40 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
