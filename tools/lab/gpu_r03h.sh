set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03h; mkdir -p $T
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dd.py tests/test_gpu_configs.py -k "dd or c4" > $T/tests.txt 2>&1 || { tail -30 $T/tests.txt; exit 1; }
tail -2 $T/tests.txt
timeout -k 10 600 python3 -u tools/dd_projection.py --n 8192 --steps 30 --ld 4 --out $T/dd_projection.json > $T/dd_projection.txt 2>&1 || { tail $T/dd_projection.txt; exit 1; }
cat $T/dd_projection.txt
