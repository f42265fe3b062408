# (historical record: written for the former FEANET_LIB_OVERRIDE variable; run variant builds through tools/lab/with_lib.py now)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; T=gpurun_out/tail2; mkdir -p $T
timeout -k 10 120 python tools/lab/tail_lab.py > $T/tail.txt 2>&1 || { cat $T/tail.txt; exit 1; }
FEANET_LIB_OVERRIDE=tools/lab/lib_old.so timeout -k 10 200 python tools/lab/tail_ab.py /tmp/ref.npz > $T/ab.txt 2>&1 || { cat $T/ab.txt; exit 1; }
timeout -k 10 200 python tools/lab/tail_ab.py /tmp/new.npz /tmp/ref.npz >> $T/ab.txt 2>&1; cat $T/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tail or vcycle" > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -2 $T/pytest.log
for i in 1 2; do
FEANET_LIB_OVERRIDE=tools/lab/lib_old.so timeout -k 10 120 python bench.py --steps 1000 --warmup 5 --no-cpu-baseline --kernel-reps 3 > $T/b_old$i.json 2>/dev/null
timeout -k 10 120 python bench.py --steps 1000 --warmup 5 --no-cpu-baseline --kernel-reps 3 > $T/b_new$i.json 2>/dev/null
done
python3 -c "
import json
for f in ['b_old1','b_new1','b_old2','b_new2']:
    print(f, json.load(open('$T/'+f+'.json'))['ms_per_step']*1e3)
"
cat $T/tail.txt
