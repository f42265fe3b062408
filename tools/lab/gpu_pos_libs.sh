# per-position cycle traces of library variants (metric configuration): bash tools/lab/gpu_pos_libs.sh TAG LIB...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp
NLINES=1 bash tools/lab/gpu_trace_libs.sh "$@" || exit 1
T=gpurun_out/$1; shift; i=0
for L in "$@"; do i=$((i+1)); echo "== $L"; python3 tools/cycle_positions.py $T/v$i; done
