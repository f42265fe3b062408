# A/B of the fine-level kernels between environment settings of the in-tree library (GPU box):
#   bash tools/lab/ab_env.sh "FEANET_BALANCE=0" ["FEANET_X=..." ...]
set -e
cd ${GRAFT_REPO_ROOT:-.}
for rep in 1 2 3; do
  echo "== A (defaults)"; timeout -k 10 120 python3 tools/lab/kern_mix.py
  for v in "$@"; do echo "== $v"; env $v timeout -k 10 120 python3 tools/lab/kern_mix.py; done
done
