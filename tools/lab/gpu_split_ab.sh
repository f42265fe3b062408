# join split A/B: parity with the in-tree build, metric cycle positions and C5 / C3 / C2 cycles against tools/lab/lib_prev.so
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_mg.py tests/test_gpu_configs.py tests/test_gpu_dd.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
bash tools/lab/gpu_pos_libs.sh $1/pos tools/lab/lib_prev.so - || exit 1
for i in 1 2; do for L in tools/lab/lib_prev.so -; do
  for cfg in "c5:--n 1024 --batch 256 --dtype f32 --steps 30 --warmup 2" "c3:--n 2048 --problem interface --steps 200" "c2:--n 1024 --levels 6 --steps 300"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 300 python3 tools/lab/with_lib.py $L bench.py --no-cpu-baseline --kernel-reps 3 $args > $T/b.json 2> $T/b.err || { tail $T/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$T/b.json')); print('$name $L', round(d['ms_per_step']*1e3,1), 'us', 'join', round(d['roofline']['avg_launch_us'],1))"
  done
done; done
