set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_mg.py -q -m gpu -p no:cacheprovider -k "coarse_tail or vcycle_vs_oracle" > gpurun_out/t_tail.log 2>&1
echo "tests rc=$?"
