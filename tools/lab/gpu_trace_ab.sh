# (historical record: written for the former FEANET_LIB_OVERRIDE variable; run variant builds through tools/lab/with_lib.py now)
# Kernel-trace A/B of the V-cycle between the in-tree library and tools/lab/lib_old.so (GPU box):
#   bash tools/lab/gpu_trace_ab.sh TAG [bench args]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
for v in old new old2 new2; do
  if [ "${v#old}" != "$v" ]; then export FEANET_LIB_OVERRIDE=tools/lab/lib_old.so; else unset FEANET_LIB_OVERRIDE; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $T/$v -o run -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --kernel-reps 2 "$@" > $T/$v.json 2> $T/$v.err || { tail $T/$v.err; exit 1; }
  python3 tools/trace_summary.py $T/$v > $T/$v.txt
  echo "== $v $(python3 -c "import json; print(json.load(open('$T/$v.json'))['ms_per_step']*1e3)") us"; head -12 $T/$v.txt
done
