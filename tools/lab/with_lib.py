"""Run a Python script against an A/B variant build of libfeanet_hip.so (lab only; the product always loads
the in-tree library):  python3 tools/lab/with_lib.py LIB.so script.py [args ...]   ("-" = the in-tree one)."""
import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
for p in (os.path.join(ROOT, "multigrid-feanet_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)
from feanet_amd import _lib  # noqa: E402

if sys.argv[1] != "-":
    _lib.LIB = os.path.abspath(sys.argv[1])
    _hmid = _lib.hmid_lds_bytes

    def _hmid_or_none(*a):  # builds older than the HJac two-level launches: none fits
        return _hmid(*a) if hasattr(_lib.lib(), "fea_mg_hmid_lds_bytes") else -1
    _lib.hmid_lds_bytes = _hmid_or_none
sys.argv = sys.argv[2:]
sys.path.insert(0, os.path.dirname(os.path.abspath(sys.argv[0])))
runpy.run_path(sys.argv[0], run_name="__main__")
