# Round-6 (session 2): the row-wave HJac tail (k_hjac_tail_fast, one barrier per level and direction) — GPU tests of
# the learned-smoother path, then same-lease A/B against the general tail (lab build FEA_HTAIL_FAST=0) and a trace.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06b_ab4; mkdir -p $T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_hnet.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
BENCH_ARGS="--n 128 --dtype f32 --smoother hjac --steps 200" bash tools/lab/gpu_cfg_libs.sh r06b_ab4/h129 - lab_libs/htail0.so || exit 1
BENCH_ARGS="--n 4096 --smoother hjac --steps 50" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06b_ab4/h4097 - lab_libs/htail0.so || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace129 -o run -- python3 bench.py --no-cpu-baseline --kernel-reps 5 --n 128 --dtype f32 --smoother hjac --steps 200 > $T/bench129.json 2> $T/bench129.err || { tail $T/bench129.err; exit 1; }
python3 tools/trace_summary.py $T/trace129 > $T/trace129.txt && head -8 $T/trace129.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace4097 -o run -- python3 bench.py --no-cpu-baseline --kernel-reps 5 --n 4096 --smoother hjac --steps 50 > $T/bench4097.json 2> $T/bench4097.err || { tail $T/bench4097.err; exit 1; }
python3 tools/trace_summary.py $T/trace4097 > $T/trace4097.txt && head -14 $T/trace4097.txt
