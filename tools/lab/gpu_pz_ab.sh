# Prolongation + sweep of the recomputed zero-guess iterate on overlapped strips: parity tests, then
# same-lease V-cycle trace A/B vs k_mg_prolong<ZU> (FEANET_PZ_OVL=0).   bash tools/lab/gpu_pz_ab.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_mid.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
bash tools/lab/gpu_trace_env.sh $1/ab "" "FEANET_PZ_OVL=0" "" "FEANET_PZ_OVL=0" || exit 1
for i in 1 2 3 4; do python3 tools/cycle_positions.py $T/ab/v$i > $T/ab/pos$i.txt && sed -n 2,9p $T/ab/pos$i.txt; done
