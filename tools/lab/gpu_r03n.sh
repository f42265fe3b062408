# Kernel trace of the 8-rank per-rank projection (PackComm: halo pack / unpack kernels included)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03n; mkdir -p $T
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof -o run -- python3 tools/dd_projection.py --n 8192 --steps 50 --ranks 8 --ld 4 > $T/proj.txt 2>&1 || { tail -20 $T/proj.txt; exit 1; }
cat $T/proj.txt
f=$(ls $T/prof/*/run_kernel_stats.csv 2>/dev/null || ls $T/prof/run_kernel_stats.csv); head -30 $f | cut -c1-200
