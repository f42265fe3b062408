# Same-lease A/B of library builds on one bench configuration, alternating A B .. A B .. (GPU box):
#   BENCH_ARGS="--n 2048 --problem interface --steps 300" bash tools/lab/gpu_cfg_libs.sh TAG LIB...  ("-" = in-tree)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
for i in ${REPS:-1 2 3}; do for L in "$@"; do
  timeout -k 10 300 python3 tools/lab/with_lib.py $L bench.py --no-cpu-baseline --kernel-reps 5 $BENCH_ARGS > $T/b.json 2> $T/b.err || { tail $T/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$T/b.json')); print('$L', round(d['ms_per_step']*1e3,2), 'us', d['roofline']['kernel'].split(' ')[0], round(d['roofline']['avg_launch_us'],2), round(d['roofline']['frac'],3))"
done; done
