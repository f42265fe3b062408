# C4 grid on one GPU (8193^2 fp64) cycle and join: library builds A B .. A B ..   bash tools/lab/gpu_c4_libs.sh TAG LIB...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
for i in 1 2 3; do for L in "$@"; do
  timeout -k 10 300 python3 tools/lab/with_lib.py $L bench.py --n 8192 --steps 60 --warmup 3 --no-cpu-baseline --kernel-reps 5 > $T/b.json 2> $T/b.err || { tail $T/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$T/b.json')); print('$L', round(d['ms_per_step']*1e3,1), 'us', 'join', round(d['roofline']['avg_launch_us'],1), round(d['roofline']['frac'],3))"
done; done
