set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06_ab5; mkdir -p $T
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_mid.py tests/test_gpu_dd.py tests/test_gpu_bench_dd.py tests/test_gpu_configs.py tests/test_gpu_pbc_dd.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
BENCH_ARGS="--n 2048 --problem interface --steps 300" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06_ab5/c3 - MID_NODES_MULTI=300000 || exit 1
BENCH_ARGS="--n 1024 --batch 256 --dtype f32 --steps 40 --warmup 2" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06_ab5/c5 - lab_libs/jpeel0.so lab_libs/junr2.so || exit 1
BENCH_ARGS="--steps 1000" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06_ab5/metric - MID_NODES=20000 || exit 1
for fg in "" "--no-fold-gather"; do
  timeout -k 10 300 python3 tools/dd_projection.py --ranks 4,8 --ld 4,5 --steps 50 $fg > $T/dd_projection$fg.txt 2>&1 || { tail $T/dd_projection$fg.txt; exit 1; }
  echo "== fold${fg}"; grep "P=" $T/dd_projection$fg.txt
done
