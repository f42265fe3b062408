# GPU check of HEAD: full GPU suite, smoke, metric bench line (+ optional extra bench args lines via $EXTRA)
#   bash tools/gpu_check.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { tail $T/smoke.log; exit 1; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $T/bench.json 2> $T/bench.err || { tail $T/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$T/bench.json')); print('bench', d['ms_per_step']*1e3, 'us', d['roofline']['frac'], d['north_star_kernel']['frac'])"
i=0
while read -r args; do
  [ -z "$args" ] && continue; i=$((i+1))
  timeout -k 10 300 python3 bench.py --no-cpu-baseline $args > $T/extra$i.json 2> $T/extra$i.err || { tail $T/extra$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$T/extra$i.json')); print('$args', d['ms_per_step']*1e3, 'us', {k: round(v['frac'],3) for k,v in d['fine_level_kernels'].items()})"
done <<< "$EXTRA"
echo done
