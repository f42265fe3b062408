# GPU DD checks: DD + config tests, then RCCL runs with all ranks on the one GPU of the box
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
T=gpurun_out/$1
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests/test_gpu_dd.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest_dd.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest_dd.log; exit 1; }
tail -2 $T/pytest_dd.log
for g in ; do  # RCCL refuses two ranks on one GPU ("Duplicate GPU detected"): needs a multi-GPU node
  P=$(( ${g%x*} * ${g#*x} ))
  timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node $P --master-addr 127.0.0.1 --master-port 2961$P tools/rccl_dd_check.py --grid $g > $T/rccl_$g.log 2>&1 || { echo "rccl $g failed"; tail -15 $T/rccl_$g.log; exit 1; }
  grep "rccl dd" $T/rccl_$g.log
done
