"""RCCL (nccl backend) run of the domain-decomposed V-cycle with every rank on ONE GPU — the direct
device path of TorchComm (RCCL P2P on framed views, deferred level-0 halo finish, all_gather_into_tensor)
that the gloo tests cannot exercise.  Launch with torchrun (--nproc-per-node P); rank 0 compares the
assembled owned blocks with a single-GPU MultigridSolver bitwise and prints one line.
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
      tools/rccl_dd_check.py --grid 1x2
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multigrid-feanet_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--grid", default=None)
    ap.add_argument("--cycles", type=int, default=3)
    args = ap.parse_args()
    import torch.distributed as dist
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    from feanet_amd.dd import DDSolver, TorchComm, default_grid
    from feanet_amd.solver import MultigridSolver
    grid = tuple(int(x) for x in args.grid.split("x")) if args.grid else default_grid(ws)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    m, n = args.m, args.n
    f = torch.randn(1, 1, m + 1, n + 1, device="cuda", dtype=torch.float64, generator=g)
    s = DDSolver(n, m, rank, ws, comm=TorchComm(), grid=grid)
    s.set_rhs(f)
    s.load()
    s.vcycle(1)
    s.vcycle(args.cycles)
    nr = s.residual_norm()
    (y0, y1), (x0, x1), u = s.owned_block()
    blocks = [None] * ws
    dist.all_gather_object(blocks, ((y0, y1, x0, x1), u.cpu()))
    if rank == 0:
        ref = MultigridSolver(n, rows=m, dtype=torch.float64)
        ref.set_rhs(f=f)
        ref.load()
        ref.vcycle(1)
        ref.vcycle(args.cycles)
        full = ref.solution().cpu()
        ok = all(torch.equal(full[:, :, a:b, c:d], blk) for (a, b, c, d), blk in blocks)
        rn = ref.residual_norm()
        print(f"rccl dd grid={grid[0]}x{grid[1]} ranks={ws} bitwise={ok} norm_rel_err="
              f"{float(((nr - rn).abs() / rn).max()):.2e}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
