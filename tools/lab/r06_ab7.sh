set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06_ab7; mkdir -p $T
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_mid.py tests/test_gpu_dd.py tests/test_gpu_configs.py tests/test_gpu_mg.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
BENCH_ARGS="--n 2048 --problem interface --steps 300" bash tools/lab/gpu_cfg_libs.sh r06_ab7/c3 - lab_libs/tp0.so || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace_c3 -o run -- python3 bench.py --no-cpu-baseline --kernel-reps 5 --n 2048 --problem interface --steps 300 > $T/bench_c3.json 2> $T/bench_c3.err || { tail $T/bench_c3.err; exit 1; }
python3 tools/trace_summary.py $T/trace_c3 > $T/trace_c3.txt && head -14 $T/trace_c3.txt
BENCH_ARGS="--n 4096 --smoother hjac --steps 50" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06_ab7/hjac - HMID_NODES=20000 || exit 1
BENCH_ARGS="--n 128 --dtype f32 --smoother hjac --steps 200" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06_ab7/hjac129 - HMID_NODES=20000
