# Line-aligned owned strips for the level-1 zero-guess prolongation + sweep: variant bitwise test, then the
# same-lease V-cycle trace A/B FEANET_PZ_BIG=2 vs 0 (k_mg_prolong<ZU>).   bash tools/lab/gpu_pzbig_ab.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_mg.py -k "variants or transfer" -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
bash tools/lab/gpu_trace_env.sh $1/ab "FEANET_PZ_BIG=2" "FEANET_PZ_BIG=0" "FEANET_PZ_BIG=2" "FEANET_PZ_BIG=0" || exit 1
for i in 1 2 3 4; do python3 tools/cycle_positions.py $T/ab/v$i > $T/ab/pos$i.txt && sed -n 2,9p $T/ab/pos$i.txt | awk '{print $2}' | tr '\n' ' '; echo; done
