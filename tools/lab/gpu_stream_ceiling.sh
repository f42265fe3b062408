set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03b; mkdir -p $T
timeout -k 10 300 python3 -u tools/lab/stream_ceiling.py > $T/ceiling.txt 2>&1 || { tail $T/ceiling.txt; exit 1; }
i=0
for C in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum" "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY" "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $T/pmc$i -o run -- python3 tools/lab/stream_ceiling.py pmc > $T/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail $T/pmc$i.log; exit 1; }
done
echo done
