set -u
mkdir -p gpurun_out/prof1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof1/bench.log 2>&1
rc=$?; echo "rc=$rc"; ls -R gpurun_out/prof1 | head -30; exit $rc
