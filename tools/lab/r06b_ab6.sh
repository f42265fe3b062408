# Round-6 (session 2): multi-level LDS groups per direction (MID_NODES_DOWN / MID_NODES_UP) on the metric cycle, with a
# per-position trace of each plan.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06b_ab6; mkdir -p $T
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_attrs.sh r06b_ab6/metric - MID_NODES_DOWN=300000 MID_NODES_UP=300000 MID_NODES=300000 MID_NODES_DOWN=70000 || exit 1
for A in MID_NODES_DOWN=300000 MID_NODES=300000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace_$A -o run -- python3 tools/lab/with_mid.py $A bench.py --no-cpu-baseline --kernel-reps 5 --steps 1000 > $T/b_$A.json 2> $T/b_$A.err || { tail $T/b_$A.err; exit 1; }
  python3 tools/cycle_positions.py $T/trace_$A > $T/pos_$A.txt 2>&1 && cat $T/pos_$A.txt
done
