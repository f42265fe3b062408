# Multi-rank bench path rehearsal on one GPU (gloo, host-staged): the N>1 line with its dd_parity record
#   bash tools/gpu_dd_parity.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 10 --warmup 2 --backend gloo --global-n 4096 > $T/dd2.json 2> $T/dd2.err || { tail -30 $T/dd2.err; exit 1; }
python3 -c "import json; d=json.load(open('$T/dd2.json')); print('dd2', d['ms_per_step'], d['dd_parity'])"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 4 --steps 10 --warmup 2 --backend gloo --global-n 4096 > $T/dd4.json 2> $T/dd4.err || { tail -30 $T/dd4.err; exit 1; }
python3 -c "import json; d=json.load(open('$T/dd4.json')); print('dd4', d['ms_per_step'], d['dd_parity'])"
echo done
