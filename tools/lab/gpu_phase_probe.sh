# Lab: phase traces of the multi-level launches (tools/lab/mid_trace.so), and of the coarse
# tail run by 1 and by 256 workgroups at once (tools/lab/tail_lab.so).   bash tools/lab/gpu_tailup_probe.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 120 python3 tools/lab/mid_trace.py > $T/mid_trace.txt 2>&1 || { tail $T/mid_trace.txt; exit 1; }
for b in 1 256 1 256; do B=$b HT=65 NLEV=6 timeout -k 10 120 python3 tools/lab/tail_lab.py >> $T/tail_trace.txt 2>&1 || { tail $T/tail_trace.txt; exit 1; }; done
grep -v amdgpu.ids $T/mid_trace.txt $T/tail_trace.txt
