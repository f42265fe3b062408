set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06_ab3; mkdir -p $T
BENCH_ARGS="--n 4096 --smoother hjac --steps 50" bash tools/lab/gpu_cfg_libs.sh r06_ab3/hjac - lab_libs/hsmw1536.so lab_libs/hsmw1024.so || exit 1
BENCH_ARGS="--steps 1000" bash tools/lab/gpu_cfg_libs.sh r06_ab3/metric - lab_libs/bal512.so lab_libs/bal768.so || exit 1
timeout -k 10 300 python3 tools/dd_projection.py --ranks 2,4,8 --steps 50 --out $T/dd_projection.json > $T/dd_projection.txt 2>&1 || { tail $T/dd_projection.txt; exit 1; }
cat $T/dd_projection.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/dd_trace -o run -- python3 tools/dd_projection.py --ranks 8 --ld 4 --steps 50 > $T/dd_trace.log 2>&1 || { tail $T/dd_trace.log; exit 1; }
python3 tools/trace_summary.py $T/dd_trace > $T/dd_trace_summary.txt && head -30 $T/dd_trace_summary.txt
BENCH_ARGS="--n 2048 --problem interface --steps 300" REPS="1 2" bash tools/lab/gpu_cfg_libs.sh r06_ab3/c3 - lab_libs/tls0.so lab_libs/l1bal.so lab_libs/l1bal1024.so
