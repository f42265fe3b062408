# DD per-rank program at 8 ranks (4x2, Ld=4) under a kernel trace: where the projected 152 us go
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03g; mkdir -p $T
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- python3 tools/dd_projection.py --n 8192 --steps 50 --ranks 8 --ld 4 > $T/proj.txt 2>&1 || { tail $T/proj.txt; exit 1; }
python3 tools/cycle_positions.py $T/trace > $T/positions.txt; cat $T/proj.txt | tail -2; cat $T/positions.txt
