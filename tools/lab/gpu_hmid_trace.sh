set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 300 python3 tools/lab/hmid_trace.py > $T/trace.txt 2>&1 || { tail -20 $T/trace.txt; exit 1; }
cat $T/trace.txt
MINT=1 timeout -k 10 300 python3 tools/lab/hmid_trace.py > $T/trace_big.txt 2>&1 || { tail -20 $T/trace_big.txt; exit 1; }
cat $T/trace_big.txt
