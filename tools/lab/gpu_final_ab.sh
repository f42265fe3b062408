# Round checkpoint + prolongation A/B: GPU suite, smoke, bench line and kernel trace (tools/gpu_check.sh),
# then the same-lease V-cycle trace A/B of the overlapped-strip prolongation on small levels.
#   bash tools/lab/gpu_final_ab.sh TAG [bench args...]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
TAG=$1
bash tools/gpu_check.sh "$@" || exit 1
python3 tools/cycle_positions.py gpurun_out/$TAG/trace > gpurun_out/$TAG/cycle_positions.txt && sed -n 1,10p gpurun_out/$TAG/cycle_positions.txt
bash tools/lab/gpu_trace_env.sh $TAG/ab "" "FEANET_PZ_OVL=0" "" "FEANET_PZ_OVL=0" || exit 1
for i in 1 2 3 4; do python3 tools/cycle_positions.py gpurun_out/$TAG/ab/v$i > gpurun_out/$TAG/ab/pos$i.txt; done
