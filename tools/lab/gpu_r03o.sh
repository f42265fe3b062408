# Host issue time vs GPU time of the per-rank projection (is the decomposed cycle host-bound?)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03o; mkdir -p $T
timeout -k 10 300 python3 tools/dd_projection.py --n 8192 --steps 50 --ld 4 > $T/proj.txt 2>&1 || { tail -20 $T/proj.txt; exit 1; }
timeout -k 10 300 python3 tools/dd_projection.py --n 8192 --steps 50 --ld 4 --no-pack > $T/proj_nopack.txt 2>&1 || { tail -20 $T/proj_nopack.txt; exit 1; }
cat $T/proj.txt $T/proj_nopack.txt
