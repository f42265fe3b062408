# DD per-rank projection: HIP-graph segments vs eager launches (the graph boundaries cost ~8 us each)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03t; mkdir -p $T
for gm in 1 3 5 100; do
  timeout -k 10 400 python3 tools/dd_projection.py --n 8192 --steps 50 --ld 4 --graph-min $gm > $T/proj_gm$gm.txt 2>&1 || { tail $T/proj_gm$gm.txt; exit 1; }
done
grep -v amdgpu.ids $T/proj_gm*.txt | grep "P="
