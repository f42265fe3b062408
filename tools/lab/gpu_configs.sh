set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/r02c5; mkdir -p $T
for cfg in "c5:--n 1024 --batch 256 --dtype f32 --steps 50 --warmup 2" "c4one:--n 8192 --steps 50" "f32_2049:--n 2048 --dtype f32 --steps 200" "c5b16:--n 1024 --batch 16 --dtype f32 --steps 200"; do
  name=${cfg%%:*}; args=${cfg#*:}
  echo "== $name"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace_$name -o run -- python3 -u bench.py --no-cpu-baseline --kernel-reps 5 $args > $T/bench_$name.json 2> $T/bench_$name.err || { tail $T/bench_$name.err; exit 1; }
  python3 tools/trace_summary.py $T/trace_$name > $T/trace_$name.txt
  python3 -c "import json; d=json.load(open('$T/bench_$name.json')); print('$name', round(d['ms_per_step']*1e3, 1), 'us/V-cycle', '%.3g DoF/s' % d['value'], 'join frac %.3f' % d['roofline']['frac'], 'sweep frac %.3f' % d['north_star_kernel']['frac'])"
  head -14 $T/trace_$name.txt
done
