# round 3: new parity tests, the multi-rank bench path rehearsed over gloo (2 processes, one GPU), DD projection
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03e; mkdir -p $T
true
tail -3 $T/tests.txt
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 2 --backend gloo --global-n 2048 --kernel-reps 3 > $T/dd2_gloo.json 2> $T/dd2_gloo.err || { tail -20 $T/dd2_gloo.err; exit 1; }
cat $T/dd2_gloo.json
timeout -k 10 600 python3 -u tools/dd_projection.py --n 8192 --steps 30 --out $T/dd_projection.json > $T/dd_projection.txt 2>&1 || { tail $T/dd_projection.txt; exit 1; }
cat $T/dd_projection.txt
timeout -k 10 400 python3 -u tools/lab/balance_ab.py > $T/balance_ab.txt 2>&1 || { tail $T/balance_ab.txt; exit 1; }
cat $T/balance_ab.txt
