# Lab: synchronised-call cost with the default scheduling flags, with spin_wait() on torch's runtime, and with the
# system runtime's flag set before torch loads (round-5 first probe).   bash tools/lab/gpu_sync.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
for m in 0 1 2 0 1; do
  SPIN=$m timeout -k 10 120 python3 tools/lab/sync_probe.py > $T/sync_$m.txt 2>&1 || { tail $T/sync_$m.txt; exit 1; }
  echo "== SPIN=$m"; grep -v amdgpu.ids $T/sync_$m.txt
done
