set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out/r06_ab1
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_bench_dd.py tests/test_gpu_dd.py -k "bench or refusal" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_ab1/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r06_ab1/pytest.log; exit 1; }
tail -3 gpurun_out/r06_ab1/pytest.log
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_libs.sh r06_ab1/metric - lab_libs/jmw1536.so lab_libs/bal3072.so lab_libs/bal4096.so lab_libs/jmw_bal.so || exit 1
BENCH_ARGS="--n 1024 --levels 6 --steps 1000" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06_ab1/c2 - lab_libs/jmw1536.so lab_libs/jmw_bal.so || exit 1
BENCH_ARGS="--n 2048 --problem interface --steps 300" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06_ab1/c3 - lab_libs/jmw1536.so lab_libs/jmw_bal.so
