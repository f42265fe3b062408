set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; T=gpurun_out/r06b_dbg1; mkdir -p $T
timeout -k 10 200 python3 tools/lab/with_lib.py - tools/lab/htail_cmp.py $T/new.npz || exit 1
timeout -k 10 200 python3 tools/lab/with_lib.py lab_libs/htail0.so tools/lab/htail_cmp.py $T/old.npz || exit 1
python3 tools/lab/htail_cmp.py --compare $T/old.npz $T/new.npz
