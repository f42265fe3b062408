set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06_ab6; mkdir -p $T
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_attrs.sh r06_ab6/metric - MID_NODES=20000 MID_NODES=70000 || exit 1
BENCH_ARGS="--n 1024 --levels 6 --steps 1000" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06_ab6/c2 - MID_NODES=20000 || exit 1
BENCH_ARGS="--n 1024 --steps 1000" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06_ab6/c2l10 - MID_NODES=20000 || exit 1
BENCH_ARGS="--n 8192 --steps 40" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06_ab6/c4one - MID_NODES=20000 || exit 1
BENCH_ARGS="--n 1024 --batch 256 --dtype f32 --steps 40 --warmup 2" REPS="1" bash tools/lab/gpu_cfg_attrs.sh r06_ab6/c5 - MID_NODES=20000 || exit 1
for A in - MID_NODES=20000; do
  timeout -k 10 300 python3 tools/lab/with_mid.py $A tools/dd_projection.py --ranks 8 --ld 4,5 --steps 50 > $T/ddp.txt 2>&1 || { tail $T/ddp.txt; exit 1; }
  echo "== dd $A"; grep "P=" $T/ddp.txt
done
