"""A/B of the pipelined vcycle(k) block decomposition: bench.py with
  new     the product's pipe_blocks (blocks of 32 + one graph for the remainder)
  old     the round-2 binary decomposition of the remainder (graph_blocks)
  headN   a first block of N cycles, then pipe_blocks of the rest (the GPU starts on a small graph while the
          host submits the large one: ROCm's graph launch costs host time per kernel node)
  python3 tools/lab/blocks_ab.py VARIANT [bench args ...]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
for p in (os.path.join(ROOT, "multigrid-feanet_amd"), ROOT):
    sys.path.insert(0, p)
from feanet_amd.solver import MultigridSolver  # noqa: E402

v = sys.argv[1]
if v == "old":
    MultigridSolver.pipe_blocks = staticmethod(MultigridSolver.graph_blocks)
elif v.startswith("head"):
    h = int(v[4:])
    base = MultigridSolver.pipe_blocks

    def head_blocks(njoin, G, _h=h, _base=base):
        return [njoin] if njoin <= _h else [_h] + _base(njoin - _h, G)
    MultigridSolver.pipe_blocks = staticmethod(head_blocks)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
import bench  # noqa: E402

bench.main()
