set -u
mkdir -p gpurun_out
python -c "import torch; print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/env.log 2>&1
timeout -k 10 400 python -m pytest tests/test_gpu_ops.py -q -m gpu -x -p no:cacheprovider > gpurun_out/t_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests/test_gpu_mg.py -q -m gpu -x -p no:cacheprovider > gpurun_out/t_mg.log 2>&1
rc=$?; echo "mg rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
