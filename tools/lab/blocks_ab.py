"""A/B of the pipelined vcycle(k) block decomposition: bench.py with the product's pipe_blocks (one graph for
the remainder) or with the round-2 binary decomposition (graph_blocks).
  python3 tools/lab/blocks_ab.py {new|old} [bench args ...]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
for p in (os.path.join(ROOT, "multigrid-feanet_amd"), ROOT):
    sys.path.insert(0, p)
from feanet_amd.solver import MultigridSolver  # noqa: E402

if sys.argv[1] == "old":
    MultigridSolver.pipe_blocks = staticmethod(MultigridSolver.graph_blocks)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
import bench  # noqa: E402

bench.main()
