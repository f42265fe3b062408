set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp
NLINES=1 bash tools/lab/gpu_trace_env.sh tw "" "FEANET_TARGET_WAVES=1024" "FEANET_TARGET_WAVES=4096" "FEANET_TARGET_WAVES=8192" || exit 1
for i in 1 2 3 4; do python3 tools/cycle_positions.py gpurun_out/tw/v$i | sed -n 2,3p; python3 tools/cycle_positions.py gpurun_out/tw/v$i | sed -n 7,10p; done
