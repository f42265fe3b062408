set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out/r06_ab2
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_mg.py tests/test_gpu_configs.py tests/test_gpu_hnet.py tests/test_gpu_mid.py -k "join or c3 or c2 or hsweep or hjac or hmid or hnet" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_ab2/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r06_ab2/pytest.log; exit 1; }
tail -2 gpurun_out/r06_ab2/pytest.log
BENCH_ARGS="--n 4096 --smoother hjac --steps 50" bash tools/lab/gpu_cfg_libs.sh r06_ab2/hjac - lab_libs/hsin0.so || exit 1
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_libs.sh r06_ab2/metric - lab_libs/jrb64.so lab_libs/jrb88.so lab_libs/bal1536.so lab_libs/bal1024.so
