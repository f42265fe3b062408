# Same-lease A/B of MultigridSolver attribute sets on one bench configuration (GPU box):
#   BENCH_ARGS="..." bash tools/lab/gpu_cfg_attrs.sh TAG ATTRS...   ("-" = defaults; e.g. MID_NODES=70000)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
for i in ${REPS:-1 2 3}; do for A in "$@"; do
  timeout -k 10 300 python3 tools/lab/with_mid.py $A bench.py --no-cpu-baseline --kernel-reps 5 $BENCH_ARGS > $T/b.json 2> $T/b.err || { tail $T/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$T/b.json')); print('$A', round(d['ms_per_step']*1e3,2), 'us', d['roofline']['kernel'].split(' ')[0], round(d['roofline']['avg_launch_us'],2))"
done; done
