# Lab probe (round 5): synchronised-call cost, mid / tail phase traces, same-lease A/Bs on the metric bench
# (join task order: -DFEA_LAB_JREV builds; the OMZ join build tools/lab/lib_omz.so), the GPU suite's join / DD tests on the
# OMZ build, then SQ counter passes over the metric cycle's kernels.
#   bash tools/lab/gpu_probe_r05.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
PYT=$(python3 -c "import pytest, os; print(os.path.join(os.path.dirname(pytest.__file__), '__main__.py'))")
timeout -k 10 400 python3 -u tools/lab/with_lib.py tools/lab/lib_omz.so $PYT tests/test_gpu_mg.py tests/test_gpu_dd.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -k "join or vcycle or dd or c4 or c3 or c5 or full_size or pipelined or solve" > $T/omz_tests.log 2>&1 || { tail -30 $T/omz_tests.log; exit 1; }
tail -2 $T/omz_tests.log
timeout -k 10 120 python3 tools/lab/sync_probe.py > $T/sync.txt 2>&1 || { tail $T/sync.txt; exit 1; }
SPIN=1 timeout -k 10 120 python3 tools/lab/sync_probe.py > $T/sync_spin.txt 2>&1 || { tail $T/sync_spin.txt; exit 1; }
cat $T/sync.txt $T/sync_spin.txt | grep -v amdgpu.ids
timeout -k 10 120 python3 tools/lab/mid_trace.py > $T/mid_trace.txt 2>&1 || { tail $T/mid_trace.txt; exit 1; }
HT=65 NLEV=6 timeout -k 10 120 python3 tools/lab/tail_lab.py > $T/tail_trace.txt 2>&1 || { tail $T/tail_trace.txt; exit 1; }
grep -v amdgpu.ids $T/mid_trace.txt $T/tail_trace.txt
for i in 1 2; do
  for v in base omz rev; do
    unset FEA_LAB_JREV; L=-
    [ $v = rev ] && export FEA_LAB_JREV=1
    [ $v = omz ] && L=tools/lab/lib_omz.so
    timeout -k 10 200 python3 tools/lab/with_lib.py $L bench.py --no-cpu-baseline --kernel-reps 5 > $T/ab_${v}_$i.json 2> $T/ab_${v}_$i.err || { tail $T/ab_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$T/ab_${v}_$i.json')); print('$v run$i', round(d['ms_per_step']*1e3,2), 'us, join', round(d['roofline']['avg_launch_us'],2), 'sweep', round(d['north_star_kernel']['avg_launch_us'],2))"
  done
done
unset FEA_LAB_JREV
P="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --kernel-reps 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $T/pmc1 -o pmc1 --output-format csv -- $P > $T/pmc1.log 2>&1 || { tail $T/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY -d $T/pmc2 -o pmc2 --output-format csv -- $P > $T/pmc2.log 2>&1 || { tail $T/pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA -d $T/pmc3 -o pmc3 --output-format csv -- $P > $T/pmc3.log 2>&1 || { tail $T/pmc3.log; exit 1; }
python3 tools/pmc_table.py $(ls $T/pmc*/*counter_collection.csv) > $T/sq_table.txt
echo done
