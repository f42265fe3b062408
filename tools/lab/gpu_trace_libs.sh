# Kernel-trace A/B of the V-cycle between library builds (GPU box):
#   bash tools/lab/gpu_trace_libs.sh TAG LIB1 LIB2 ...   ("-" = the in-tree library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
i=0
for L in "$@"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $T/v$i -o run -- python3 tools/lab/with_lib.py $L bench.py --steps 300 --warmup 5 --no-cpu-baseline --kernel-reps 2 $BENCH_ARGS > $T/v$i.json 2> $T/v$i.err || { tail $T/v$i.err; exit 1; }
  python3 tools/trace_summary.py $T/v$i > $T/v$i.txt
  echo "== [$L] $(python3 -c "import json; print(json.load(open('$T/v$i.json'))['ms_per_step']*1e3)") us"; head -${NLINES:-9} $T/v$i.txt
done
