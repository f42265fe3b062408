# Round profile (PMC passes, bench line, its kernel trace and per-position view) and every BASELINE
# configuration's kernel trace, in one GPU call:   bash tools/gpu_final.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp
bash tools/profile_round.sh $1 || exit 1
python3 tools/cycle_positions.py gpurun_out/$1/trace > gpurun_out/$1/cycle_positions.txt && cat gpurun_out/$1/cycle_positions.txt
bash tools/gpu_configs.sh $1_configs || exit 1
