# Round-6 (session 2) A/B: join tasks flip their streaming direction every launch (lab_libs/jflip.so) vs HEAD.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06b_ab1; mkdir -p $T
for L in - lab_libs/jflip.so; do
  timeout -k 10 200 python3 tools/lab/with_lib.py $L tools/lab/lib_hash.py 4096 37 > $T/hash_$(basename $L).txt 2> $T/hash.err || { tail $T/hash.err; exit 1; }
  cat $T/hash_$(basename $L).txt
done
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_libs.sh r06b_ab1/metric - lab_libs/jflip.so || exit 1
BENCH_ARGS="--n 2048 --problem interface --steps 300" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06b_ab1/c3 - lab_libs/jflip.so || exit 1
BENCH_ARGS="--n 8192 --steps 100" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06b_ab1/c4 - lab_libs/jflip.so || exit 1
