set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_mg.py -q -m gpu -x -p no:cacheprovider > gpurun_out/t_mg2.log 2>&1
rc=$?; echo "mg rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench2.log 2>&1
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p gpurun_out/prof2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof2/bench.log 2>&1
echo "prof rc=$?"
