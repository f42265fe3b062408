# MG-HJac 4097^2 fp64 cycle: library builds A B .. A B .., then a kernel trace of each
#   bash tools/lab/gpu_hjac_libs.sh TAG LIB1 LIB2 ...   ("-" = the in-tree library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
for i in 1 2; do for L in "$@"; do
  timeout -k 10 300 python3 tools/lab/with_lib.py $L bench.py --smoother hjac --steps 200 --warmup 5 --no-cpu-baseline --kernel-reps 3 > $T/b.json 2> $T/b.err || { tail $T/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$T/b.json')); print('$L', round(d['ms_per_step']*1e3,1), 'us')"
done; done
i=0
for L in "$@"; do i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/v$i -o run -- python3 tools/lab/with_lib.py $L bench.py --smoother hjac --steps 200 --warmup 5 --no-cpu-baseline --kernel-reps 3 > $T/v$i.json 2> $T/v$i.err || { tail $T/v$i.err; exit 1; }
  python3 tools/trace_summary.py $T/v$i > $T/v$i.txt; echo "== $L"; head -9 $T/v$i.txt
done
