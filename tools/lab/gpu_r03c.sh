# round-3 lab: same-process A/B of nontemporal f/u loads (lib_ntl.so) + C5 join knobs; SQ counters of the C5 join
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r03c; mkdir -p $T
timeout -k 10 400 python3 -u tools/lab/ntl_ab.py tools/lab/lib_ntl.so > $T/ntl_ab.txt 2>&1 || { tail $T/ntl_ab.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $T/sq -o run -- python3 bench.py --n 1024 --batch 256 --dtype f32 --no-cpu-baseline --steps 3 --warmup 1 --kernel-reps 1 > $T/sq.log 2>&1 || { echo "pmc failed"; tail $T/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $T/sq64 -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --kernel-reps 1 > $T/sq64.log 2>&1 || { echo "pmc failed"; tail $T/sq64.log; exit 1; }
python3 tools/pmc_table.py $T/sq/*counter_collection.csv > $T/sq.txt; python3 tools/pmc_table.py $T/sq64/*counter_collection.csv > $T/sq64.txt
echo done
