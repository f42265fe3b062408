# vcycle(k) block decomposition A/B at the driver's step count (bench.py --steps 20 --warmup 5), alternating
#   bash tools/lab/gpu_blocks_ab.sh TAG VARIANT [VARIANT ...]     (variants: tools/lab/blocks_ab.py)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
for rep in 1 2 3; do
  for v in "$@"; do
    timeout -k 10 300 python3 tools/lab/blocks_ab.py $v --steps 20 --warmup 5 --no-cpu-baseline --kernel-reps 5 > $T/$v$rep.json 2> $T/$v.err || { tail $T/$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$T/$v$rep.json')); print('$v', round(d['ms_per_step']*1e3,2), 'us')"
  done
done
