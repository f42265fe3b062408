# Every BASELINE configuration (+ the learned-smoother cycle) through bench.py under a kernel trace:
#   bash tools/gpu_configs.sh TAG [names...]       (GPU box; records under gpurun_out/TAG)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
ALL="c2:--n 1024 --levels 6 --steps 200
c2l10:--n 1024 --steps 200
c3:--n 2048 --problem interface --steps 100
c4one:--n 8192 --steps 40
c5:--n 1024 --batch 256 --dtype f32 --steps 40 --warmup 2
hjac129:--n 128 --dtype f32 --smoother hjac --steps 200
hjac4097:--n 4096 --smoother hjac --steps 20"
while IFS= read -r cfg; do
  name=${cfg%%:*}; args=${cfg#*:}
  if [ $# -gt 0 ] && ! printf '%s\n' "$@" | grep -qx "$name"; then continue; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace_$name -o run -- python3 -u bench.py --no-cpu-baseline --kernel-reps 5 $args > $T/bench_$name.json 2> $T/bench_$name.err || { tail $T/bench_$name.err; exit 1; }
  python3 tools/trace_summary.py $T/trace_$name > $T/trace_$name.txt
  python3 -c "import json; d=json.load(open('$T/bench_$name.json')); print('$name', round(d['ms_per_step']*1e3, 1), 'us/V-cycle', '%.3g DoF/s' % d['value'], 'join frac %.3f' % d['roofline']['frac'], 'sweep frac %.3f' % d['north_star_kernel']['frac'])"
done <<< "$ALL"
