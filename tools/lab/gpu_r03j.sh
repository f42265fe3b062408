set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03j; mkdir -p $T
timeout -k 10 300 python3 -u tools/lab/hsweep_ab.py > $T/hsweep_ab.txt 2>&1 || { tail -20 $T/hsweep_ab.txt; exit 1; }
cat $T/hsweep_ab.txt
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hnet.py > $T/tests.txt 2>&1 || { tail -30 $T/tests.txt; exit 1; }
tail -2 $T/tests.txt
bash tools/gpu_configs.sh r03j hjac129 hjac4097
