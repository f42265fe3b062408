# Round-6 (session 2): the tail extended by the level above it (fea_mg_coarse_tail_ext) — GPU tests, then
# same-lease A/B TAIL_EXT on (default) / off on the metric, C2 and C5 configurations, and a kernel trace.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06b_ab2; mkdir -p $T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mg.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tail_ext or coarse_tail_kernel or joined_vcycles or full_size_vs_oracle or pairs_restrictions or vcycle_vs_oracle" > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_attrs.sh r06b_ab2/metric - TAIL_EXT=0 || exit 1
BENCH_ARGS="--n 1024 --levels 6 --steps 1000" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06b_ab2/c2 - TAIL_EXT=0 || exit 1
BENCH_ARGS="--n 1024 --dtype f32 --batch 256 --steps 40" REPS="1 2" bash tools/lab/gpu_cfg_attrs.sh r06b_ab2/c5 - TAIL_EXT=0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o run -- python3 bench.py --no-cpu-baseline --kernel-reps 5 --steps 1000 > $T/bench.json 2> $T/bench.err || { tail $T/bench.err; exit 1; }
python3 tools/trace_summary.py $T/trace > $T/trace.txt && head -12 $T/trace.txt
python3 tools/cycle_positions.py $T/trace > $T/positions.txt 2>&1 && head -12 $T/positions.txt
