# PMC passes (HBM traffic + SQ instruction / wait counters) for bench configurations, one rocprofv3 pass per
# counter group (GPU box):   bash tools/lab/gpu_cfg_pmc.sh TAG name...   (names: c3 p2049 c5 metric hjac)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/$1; shift; mkdir -p $T
declare -A CFG=(
  [c3]="--n 2048 --problem interface --steps 20"
  [p2049]="--n 2048 --steps 20"
  [c5]="--n 1024 --batch 256 --dtype f32 --steps 5 --warmup 1"
  [metric]="--steps 20"
  [hjac]="--n 4096 --smoother hjac --steps 5"
)
PASSES=("FETCH_SIZE" "WRITE_SIZE"
        "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE")
for name in "$@"; do
  i=0
  for P in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $T/${name}_p$i -o run -- python3 bench.py --no-cpu-baseline --kernel-reps 3 ${CFG[$name]} > $T/${name}_p$i.log 2>&1 || { echo "pmc $name pass $i failed"; tail -5 $T/${name}_p$i.log; exit 1; }
    echo "$name pass $i ok"
  done
  python3 tools/pmc_table.py $T/${name}_p*/*counter_collection.csv > $T/${name}_table.txt
  python3 tools/pmc_traffic.py $(ls $T/${name}_p1/*counter_collection.csv) $(ls $T/${name}_p2/*counter_collection.csv) $T/${name}_traffic.json $T/${name}_traffic.txt > /dev/null
  head -8 $T/${name}_traffic.txt
done
# keep the summaries only (the raw csv of a pass is tens of MB; gpurun copies back <= 64 MiB)
rm -rf $T/*_p[0-9]
