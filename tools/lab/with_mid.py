"""Lab: run a script with MultigridSolver class attributes overridden (plan A/B without a rebuild):
    python3 tools/lab/with_mid.py MID_NODES=70000[,MID_MIN_TILES=...] script.py [args ...]"""
import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
for p in (os.path.join(ROOT, "multigrid-feanet_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)
from feanet_amd.solver import MultigridSolver  # noqa: E402

for kv in sys.argv[1].split(","):
    if kv and kv != "-":
        k, v = kv.split("=")
        old = getattr(MultigridSolver, k)
        if isinstance(old, bool):
            v = v not in ("0", "False", "false")
        elif old is None:
            v = int(v)
        else:
            v = type(old)(v)
        setattr(MultigridSolver, k, v)
sys.argv = sys.argv[2:]
sys.path.insert(0, os.path.dirname(os.path.abspath(sys.argv[0])))
runpy.run_path(sys.argv[0], run_name="__main__")
