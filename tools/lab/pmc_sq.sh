cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU -d gpurun_out/pmc1 -o pmc1 --output-format csv -- python3 tools/lab/kern_mix.py > gpurun_out/pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc2 -o pmc2 --output-format csv -- python3 tools/lab/kern_mix.py > gpurun_out/pmc2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc3 -o pmc3 --output-format csv -- python3 tools/lab/kern_mix.py > gpurun_out/pmc3.log 2>&1
echo rc=$?
