# Round-6 (session 3): fp64 two-material coarse tail with float-exact tables staged as float (FEA_TAIL_F32_TABLES) —
# tail tests, bitwise hash flag on / off at C3, same-lease A/B on C3, a C3 trace.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06c_f32tab; mkdir -p $T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mg.py -m gpu -x -q --timeout 300 --timeout-method thread -k "coarse_tail or interface" > $T/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
for A in TAIL_F32_TABLES=1 TAIL_F32_TABLES=0; do
  timeout -k 10 200 python3 tools/lab/with_mid.py $A tools/lab/lib_hash.py 2048 37 interface > $T/hash.txt 2> $T/hash.err || { tail $T/hash.err; exit 1; }
  echo "$A $(cat $T/hash.txt)"
done
BENCH_ARGS="--n 2048 --problem interface --steps 300" bash tools/lab/gpu_cfg_attrs.sh r06c_f32tab/c3 TAIL_F32_TABLES=1 TAIL_F32_TABLES=0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace_c3 -o run -- python3 bench.py --no-cpu-baseline --kernel-reps 5 --n 2048 --problem interface --steps 300 > $T/bench_c3.json 2> $T/bench_c3.err || { tail $T/bench_c3.err; exit 1; }
python3 tools/cycle_positions.py $T/trace_c3 > $T/positions_c3.txt 2>&1 && cat $T/positions_c3.txt
