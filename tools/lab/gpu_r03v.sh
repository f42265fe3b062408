# Uniform-task path of the two-material join: GPU suite, C3 A/B against the all-indexed build, dd parity rehearsal
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/${1:-r03v}; mkdir -p $T
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
for rep in 1 2; do
  for lib in - ${LIBB:-tools/lab/lib_head.so} $LIBC; do
    timeout -k 10 300 python3 tools/lab/with_lib.py $lib bench.py --n 2048 --problem interface --steps 200 --warmup 5 --no-cpu-baseline > $T/c3_$rep$(basename $lib).json 2> $T/c3.err || { tail $T/c3.err; exit 1; }
    python3 -c "import json; d=json.load(open('$T/c3_$rep$(basename $lib).json')); print('$lib', round(d['ms_per_step']*1e3,2), 'us', {k: round(v['avg_launch_us'],2) for k,v in d['fine_level_kernels'].items()})"
  done
done
[ -n "$2" ] && bash tools/gpu_dd_parity.sh ${1}_ddp; echo end
if [ -n "$TRACE" ]; then
  for lib in - ${LIBB:-tools/lab/lib_head.so} $LIBC; do
    nm=$(basename $lib)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace_c3$nm -o run -- python3 tools/lab/with_lib.py $lib bench.py --n 2048 --problem interface --steps 200 --warmup 5 --no-cpu-baseline > $T/trace_c3$nm.json 2> $T/trace_c3$nm.err || { tail $T/trace_c3$nm.err; exit 1; }
    python3 tools/trace_summary.py $T/trace_c3$nm > $T/trace_c3$nm.txt && head -9 $T/trace_c3$nm.txt
  done
fi
