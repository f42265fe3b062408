set -u
mkdir -p gpurun_out/prof4
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 50 --warmup 5 > gpurun_out/prof4/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4/trace -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof4/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof4/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --kernel-reps 10 > gpurun_out/prof4/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof4/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --kernel-reps 10 > gpurun_out/prof4/pmc_write.log 2>&1
echo "write rc=$?"
