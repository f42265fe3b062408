set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp
BENCH_ARGS="--n 2048 --problem interface --steps 300" bash tools/lab/gpu_cfg_attrs.sh r06_ab4/c3 - MID_NODES=70000 MID_NODES=20000 || exit 1
BENCH_ARGS="--steps 1000" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06_ab4/metric - MID_NODES=70000 || exit 1
BENCH_ARGS="--n 1024 --levels 6 --steps 1000" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06_ab4/c2 - MID_NODES=70000
