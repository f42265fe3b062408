# A/B of the whole V-cycle (bench.py ms_per_step) between environment settings (GPU box):
#   bash tools/lab/ab_bench.sh "FEANET_TARGET_WAVES=4096" ["FEANET_X=..." ...]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
run() { env "$@" timeout -k 10 120 python3 bench.py --steps ${STEPS:-1000} --warmup 5 --no-cpu-baseline --kernel-reps 3 \
          | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f us' % (d['ms_per_step']*1e3))"; }
for rep in 1 2 3; do
  echo "== defaults: $(run A=1)" || exit 1
  for v in "$@"; do echo "== $v: $(run $v)" || exit 1; done
done
