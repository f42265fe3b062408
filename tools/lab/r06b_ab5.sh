# Round-6 (session 2): two-material stiffness taps from the centre's table row (FEA_KSYM=1, bitwise) — GPU tests of the
# two-material paths, bitwise hash vs the tap-pattern build, same-lease A/B on C3 and a C3 trace.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06b_ab5; mkdir -p $T
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_mg.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "interface or c3 or C3" > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
for L in - lab_libs/ksym0.so; do
  timeout -k 10 200 python3 tools/lab/with_lib.py $L tools/lab/lib_hash.py 2048 37 interface > $T/hash.txt 2> $T/hash.err || { tail $T/hash.err; exit 1; }
  echo "$L $(cat $T/hash.txt)"
done
BENCH_ARGS="--n 2048 --problem interface --steps 300" bash tools/lab/gpu_cfg_libs.sh r06b_ab5/c3 - lab_libs/ksym0.so || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace_c3 -o run -- python3 bench.py --no-cpu-baseline --kernel-reps 5 --n 2048 --problem interface --steps 300 > $T/bench_c3.json 2> $T/bench_c3.err || { tail $T/bench_c3.err; exit 1; }
python3 tools/trace_summary.py $T/trace_c3 > $T/trace_c3.txt && head -10 $T/trace_c3.txt
python3 tools/cycle_positions.py $T/trace_c3 > $T/positions_c3.txt 2>&1 && cat $T/positions_c3.txt
