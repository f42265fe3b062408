# Round checkpoint on the GPU box: GPU suite, smoke, the round profile (PMC passes + bench line + kernel
# trace, tools/profile_round.sh), and kernel traces of the other BASELINE configurations.
#   bash tools/gpu_round.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
TAG=$1
T=gpurun_out/$TAG
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest_gpu.log; exit 1; }
tail -1 $T/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { cat $T/smoke.log; exit 1; }
tail -1 $T/smoke.log
bash tools/profile_round.sh $TAG || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $T/bench_steps20.json 2> $T/bench_steps20.err || { tail $T/bench_steps20.err; exit 1; }
for cfg in "c2:--n 1024 --steps 300" "c3:--n 2048 --problem interface --steps 300" "c5:--n 1024 --batch 256 --dtype f32 --steps 30 --warmup 2" "c4one:--n 8192 --steps 50" "f32_2049:--n 2048 --dtype f32 --steps 300"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace_$name -o run -- python3 bench.py --no-cpu-baseline --kernel-reps 5 $args > $T/bench_$name.json 2> $T/bench_$name.err || { tail $T/bench_$name.err; exit 1; }
  python3 tools/trace_summary.py $T/trace_$name > $T/trace_$name.txt
  python3 -c "import json; d=json.load(open('$T/bench_$name.json')); print('$name', round(d['ms_per_step']*1e3, 1), 'us/V-cycle', '%.3g DoF/s' % d['value'], 'join frac %.3f' % d['roofline']['frac'], 'sweep frac %.3f' % d['north_star_kernel']['frac'])"
done
