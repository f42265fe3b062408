# Lab probe (round 5): same-lease A/B of the join's alternating task order (FEA_LAB_JREV) on the metric
# bench, then SQ counter passes over the metric cycle's kernels.
#   bash tools/lab/gpu_probe_r05.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
for i in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export FEA_LAB_JREV=1; else unset FEA_LAB_JREV; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --kernel-reps 5 > $T/ab_rev${v}_$i.json 2> $T/ab_rev${v}_$i.err || { tail $T/ab_rev${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$T/ab_rev${v}_$i.json')); print('rev$v run$i', round(d['ms_per_step']*1e3,2), 'us, join', round(d['roofline']['avg_launch_us'],2))"
  done
done
unset FEA_LAB_JREV
P="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --kernel-reps 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $T/pmc1 -o pmc1 --output-format csv -- $P > $T/pmc1.log 2>&1 || { tail $T/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY -d $T/pmc2 -o pmc2 --output-format csv -- $P > $T/pmc2.log 2>&1 || { tail $T/pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA -d $T/pmc3 -o pmc3 --output-format csv -- $P > $T/pmc3.log 2>&1 || { tail $T/pmc3.log; exit 1; }
python3 tools/pmc_table.py $(ls $T/pmc*/*counter_collection.csv) > $T/sq_table.txt
echo done
