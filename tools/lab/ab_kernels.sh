# (historical record: written for the former FEANET_LIB_OVERRIDE variable; run variant builds through tools/lab/with_lib.py now)
# A/B of the fine-level kernels between the in-tree library and variant libraries (GPU box):
#   bash tools/lab/ab_kernels.sh tools/lab/libB.so [tools/lab/libC.so ...]
# Alternates processes A, B, ... three times each; each prints per-kernel times (kern_mix.py).
set -e
cd ${GRAFT_REPO_ROOT:-.}
for rep in 1 2 3; do
  echo "== A (in-tree)"; timeout -k 10 120 python3 tools/lab/kern_mix.py
  for v in "$@"; do echo "== $v"; FEANET_LIB_OVERRIDE=$v timeout -k 10 120 python3 tools/lab/kern_mix.py; done
done
