# One-call A/B on the GPU box: GPU tests of a selection, then per-position cycle traces of the library builds
# twice in alternation (A B .. A B ..), then the PMC traffic passes of each build.
#   bash tools/lab/gpu_ab.sh TAG "pytest selection or -" LIB1 LIB2 ...   ("-" = the in-tree library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; TAG=$1; SEL=$2; shift 2; T=gpurun_out/$TAG; mkdir -p $T
if [ "$SEL" != "-" ]; then
  timeout -k 10 600 python3 -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $T/pytest.log; exit 1; }
  tail -1 $T/pytest.log
fi
bash tools/lab/gpu_pos_libs.sh $TAG/pos1 "$@" || exit 1
bash tools/lab/gpu_pos_libs.sh $TAG/pos2 "$@" || exit 1
[ -n "$NO_PMC" ] || bash tools/lab/gpu_pmc_libs.sh $TAG/pmc "$@" || exit 1
