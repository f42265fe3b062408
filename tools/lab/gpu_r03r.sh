# A/B of the fused restriction's wave target (2048 default / 4096 / 8192 waves)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03r; mkdir -p $T
for L in - tools/lab/lib_zr2_w4096.so tools/lab/lib_zr2_w8192.so; do
  timeout -k 10 300 python3 tools/lab/with_lib.py $L tools/lab/zr2_ab.py >> $T/zr2_ab.txt 2>&1 || { tail -20 $T/zr2_ab.txt; exit 1; }
done
cat $T/zr2_ab.txt | grep -v amdgpu.ids
