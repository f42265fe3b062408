# Round-6 (session 2): the fp64 join's 4-row prefetch ring (FEA_JOIN_AHEAD=4, 163 VGPRs, no spills) now that the
# launch holds ~2 waves per SIMD (1536-wave minimum) — bitwise hash, same-lease A/B on metric, C2, C4 grid.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06b_ab7; mkdir -p $T
for L in - lab_libs/jahead4.so; do
  timeout -k 10 200 python3 tools/lab/with_lib.py $L tools/lab/lib_hash.py 4096 37 > $T/hash.txt 2> $T/hash.err || { tail $T/hash.err; exit 1; }
  echo "$L $(cat $T/hash.txt)"
done
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_libs.sh r06b_ab7/metric - lab_libs/jahead4.so || exit 1
BENCH_ARGS="--n 1024 --levels 6 --steps 1000" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06b_ab7/c2 - lab_libs/jahead4.so || exit 1
BENCH_ARGS="--n 8192 --steps 100" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06b_ab7/c4 - lab_libs/jahead4.so || exit 1
