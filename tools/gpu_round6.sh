# Round-6 evidence, part 1 (GPU box): full GPU suite, smoke, the round profile (PMC traffic passes, the bench line and
# its kernel trace: tools/profile_round.sh), per-position cycle view, bench --steps 20.   bash tools/gpu_round6.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; TAG=$1; T=gpurun_out/$TAG; mkdir -p $T
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest_gpu.log; exit 1; }
tail -1 $T/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { cat $T/smoke.log; exit 1; }
tail -1 $T/smoke.log
bash tools/profile_round.sh $TAG || exit 1
python3 tools/cycle_positions.py $T/trace > $T/cycle_positions.txt && cat $T/cycle_positions.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $T/bench_steps20.json 2> $T/bench_steps20.err || { tail $T/bench_steps20.err; exit 1; }
python3 -c "import json; d=json.load(open('$T/bench_steps20.json')); print('steps20', round(d['ms_per_step']*1e3, 2), 'us')"
