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
    # an older build: bind only what it exports, and keep the solver off the entry points it lacks
    import ctypes
    _L = ctypes.CDLL(_lib.LIB)
    for base in list(_lib._SIGS):
        if not hasattr(_L, f"fea_{base}_f64"):
            del _lib._SIGS[base]
    for name in list(_lib._EXTRA):
        if not hasattr(_L, name):
            del _lib._EXTRA[name]
    if not hasattr(_L, "fea_mg_tail_up_f64"):
        from feanet_amd import solver as _solver
        _solver.MultigridSolver._can_tail_up = lambda self, *a: False
sys.argv = sys.argv[2:]
sys.path.insert(0, os.path.dirname(os.path.abspath(sys.argv[0])))
runpy.run_path(sys.argv[0], run_name="__main__")
