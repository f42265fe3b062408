set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/lab/tail_lab.py && MULTI=1 timeout -k 10 120 python3 tools/lab/tail_lab.py
