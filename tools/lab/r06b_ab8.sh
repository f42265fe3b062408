# Round-6 (session 2): framed row pitch + 1 / + 5 128-byte lines (lab FEA_LAB_LD_PAD) on the metric and the C4 grid.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06b_ab8; mkdir -p $T
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_libs.sh r06b_ab8/metric - lab_libs/ldpad1.so lab_libs/ldpad5.so || exit 1
BENCH_ARGS="--n 8192 --steps 100" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06b_ab8/c4 - lab_libs/ldpad1.so lab_libs/ldpad5.so || exit 1
