# One-phase DD halo exchange (packed staging, fea_dd_copy_blocks): DD + config parity, gloo bench rehearsal
# over 2 and 4 ranks (2x1 slabs, 2x2 blocks), per-rank projection with the pack / unpack kernels
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03m; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_gpu_dd.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $T/pytest_dd.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest_dd.log; exit 1; }
tail -2 $T/pytest_dd.log
for P in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $P --master-addr 127.0.0.1 --master-port 2957$P bench.py --gpus $P --steps 10 --warmup 2 --backend gloo --global-n 2048 --kernel-reps 3 > $T/dd${P}_gloo.json 2> $T/dd${P}_gloo.err || { tail -20 $T/dd${P}_gloo.err; exit 1; }
  cat $T/dd${P}_gloo.json
done
timeout -k 10 400 python3 tools/dd_projection.py --n 8192 --steps 50 --ld 3,4,5 --out $T/dd_projection.json > $T/dd_projection.txt 2>&1 || { tail -20 $T/dd_projection.txt; exit 1; }
cat $T/dd_projection.txt
timeout -k 10 400 python3 tools/dd_projection.py --n 8192 --steps 50 --ld 4 --no-pack > $T/dd_projection_nopack.txt 2>&1 || { tail -20 $T/dd_projection_nopack.txt; exit 1; }
cat $T/dd_projection_nopack.txt
