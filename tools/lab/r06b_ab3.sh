# Round-6 (session 2): coarse-tail workgroup size (lab builds FEA_TAIL_THREADS=512 / 256) and the tail's top size
# (MultigridSolver.TAIL_MAX_N = 33: the 65^2 level goes to the paired streaming kernels) — same-lease A/B.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06b_ab3; mkdir -p $T
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mg.py -m gpu -x -q --timeout 120 --timeout-method thread -k "coarse_tail_kernel" > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
for L in - lab_libs/tail512.so lab_libs/tail256.so; do
  timeout -k 10 200 python3 tools/lab/with_lib.py $L tools/lab/lib_hash.py 4096 37 > $T/hash.txt 2> $T/hash.err || { tail $T/hash.err; exit 1; }
  echo "$L $(cat $T/hash.txt)"
done
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_libs.sh r06b_ab3/threads - lab_libs/tail512.so lab_libs/tail256.so || exit 1
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_attrs.sh r06b_ab3/metric - TAIL_MAX_N=33 || exit 1
BENCH_ARGS="--n 1024 --levels 6 --steps 1000" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06b_ab3/c2 - TAIL_MAX_N=33 || exit 1
BENCH_ARGS="--n 2048 --problem interface --steps 300" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06b_ab3/c3 - TAIL_MAX_N=33 || exit 1
BENCH_ARGS="--n 1024 --dtype f32 --batch 256 --steps 40" REPS="1" bash tools/lab/gpu_cfg_attrs.sh r06b_ab3/c5 - TAIL_MAX_N=33 || exit 1
BENCH_ARGS="--n 2048 --problem interface --steps 300" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06b_ab3/c3threads - lab_libs/tail512.so || exit 1
