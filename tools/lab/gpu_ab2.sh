# A/B of variant libraries on the metric configuration and C5 (same lease, alternating processes)
#   bash tools/lab/gpu_ab2.sh TAG LIB [LIB ...]       ("-" = the in-tree library)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
for rep in 1 2; do
  for lib in "$@"; do
    nm=$(basename $lib)
    timeout -k 10 300 python3 tools/lab/with_lib.py $lib bench.py --steps 200 --warmup 5 --no-cpu-baseline --kernel-reps 10 > $T/m_$rep$nm.json 2> $T/m.err || { tail $T/m.err; exit 1; }
    python3 -c "import json; d=json.load(open('$T/m_$rep$nm.json')); print('metric $lib', round(d['ms_per_step']*1e3,2), 'us join', round(d['roofline']['avg_launch_us'],2))"
    timeout -k 10 300 python3 tools/lab/with_lib.py $lib bench.py --n 1024 --batch 256 --dtype f32 --steps 20 --warmup 2 --no-cpu-baseline --kernel-reps 5 > $T/c5_$rep$nm.json 2> $T/c5.err || { tail $T/c5.err; exit 1; }
    python3 -c "import json; d=json.load(open('$T/c5_$rep$nm.json')); print('c5 $lib', round(d['ms_per_step']*1e3,1), 'us', {k: round(v['avg_launch_us'],1) for k,v in d['fine_level_kernels'].items()})"
  done
done
