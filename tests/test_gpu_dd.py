"""GPU parity of the domain-decomposed V-cycle (feanet_amd.dd): P row slabs on one device (the
in-process LocalGroup, and two processes over gloo) against the single-GPU MultigridSolver on the
same global grid.  The decomposition uses the same kernels with the same per-node arithmetic, so
the owned rows must agree bitwise (torch.equal), cycle after cycle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _global_problem(m, n, B, seed=0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    f = torch.randn(B, 1, m + 1, n + 1, device="cuda", dtype=torch.float64, generator=g)
    u0 = torch.randn(B, 1, m + 1, n + 1, device="cuda", dtype=torch.float64, generator=g)
    bc = torch.rand(B, 1, m + 1, n + 1, device="cuda", dtype=torch.float64, generator=g)
    inner = torch.zeros_like(bc)
    inner[..., 1:-1, 1:-1] = 1
    return f, u0, bc * (1 - inner)


def _single(m, n, B, f, u0, bc, cycles, nu=(1, 1)):
    from feanet_amd.solver import MultigridSolver
    s = MultigridSolver(n, rows=m, dtype=torch.float64, batch=B, nu1=nu[0], nu2=nu[1])
    s.set_boundary(bc)
    s.set_rhs(f=f)
    s.load(u0)
    out = []
    for _ in range(cycles):
        s.vcycle()
        out.append((s.solution(), s.residual_norm()))
    return s, out


@pytest.mark.parametrize("m,n,P,Ld,B,graph,nu,grid", [(256, 128, 2, 1, 1, True, (1, 1), None),
                                                      (512, 256, 4, 2, 2, True, (1, 1), None),
                                                      (384, 256, 3, 2, 1, False, (1, 1), None),
                                                      (1024, 1024, 4, 3, 1, True, (1, 1), None),
                                                      (2048, 1024, 8, 3, 1, True, (1, 1), None),
                                                      (2048, 1024, 8, 4, 1, True, (1, 1), None),
                                                      (4096, 512, 4, 5, 1, True, (1, 1), None),
                                                      (1024, 512, 4, 3, 1, True, (2, 2), None),
                                                      (1024, 512, 2, 3, 1, False, (2, 1), None),
                                                      # 2-D blocks (x-then-y exchange, corners via diagonals)
                                                      (512, 512, 4, 2, 2, True, (1, 1), (2, 2)),
                                                      (1024, 1024, 8, 3, 1, True, (1, 1), (4, 2)),
                                                      (512, 1024, 2, 3, 1, True, (1, 1), (1, 2)),
                                                      (768, 1024, 6, 2, 1, False, (1, 1), (3, 2)),
                                                      (1024, 1024, 4, 3, 1, True, (2, 2), (2, 2))])
def test_dd_local_group_bitwise(m, n, P, Ld, B, graph, nu, grid):
    """Communication-avoiding exchanges (one neighbour batch per cycle, exchange_depths): every owned
    node still equals the single-GPU V-cycle bit for bit — row slabs and 2-D blocks, also with deeper
    agglomeration and V(2,2)."""
    from feanet_amd.dd import LocalGroup
    f, u0, bc = _global_problem(m, n, B)
    s, ref = _single(m, n, B, f, u0, bc, 4, nu)
    grp = LocalGroup(n, m, P, agglomerate=Ld, batch=B, graph=graph, nu1=nu[0], nu2=nu[1], grid=grid)
    assert grp.ranks[0].coarse.tail_from is None or grp.ranks[0].coarse.tail_from + Ld == s.tail_from
    grp.set_rhs(f)
    grp.load(u0, bc)
    for k in range(4):
        grp.vcycle()
        got = grp.solution()
        assert torch.equal(got, ref[k][0]), f"cycle {k}: max diff {(got - ref[k][0]).abs().max().item():.3e}"
        nr = grp.residual_norm()
        torch.testing.assert_close(nr, ref[k][1], rtol=1e-12, atol=0)
    # several cycles per call: the finest level's cycle boundaries joined on every slab
    s.vcycle(3)
    grp.vcycle(3)
    assert torch.equal(grp.solution(), s.solution())
    s.vcycle(2)
    grp.vcycle(2)
    assert torch.equal(grp.solution(), s.solution())


def _free_port():
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    p = sk.getsockname()[1]
    sk.close()
    return p


def _dd_worker(rank, world, m, n, Ld, port, outdir, grid):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "multigrid-feanet_amd"))
    import torch.distributed as dist
    from feanet_amd.dd import DDSolver, TorchComm
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    f, u0, bc = _global_problem(m, n, 1)
    s = DDSolver(n, m, rank, world, comm=TorchComm(), agglomerate=Ld, grid=grid)
    s.set_rhs(f)
    s.load(u0, bc)
    s.vcycle(3)
    (y0, y1), (x0, x1), u = s.owned_block()
    nr = s.residual_norm()
    torch.cuda.synchronize()
    np.save(os.path.join(outdir, f"r{rank}.npy"), u.cpu().numpy())
    np.save(os.path.join(outdir, f"i{rank}.npy"), np.array([y0, y1, x0, x1]))
    np.save(os.path.join(outdir, f"n{rank}.npy"), nr.cpu().numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("m,n,P,Ld,grid", [(512, 256, 2, 2, None), (256, 512, 2, 2, (1, 2)), (512, 512, 4, 2, (2, 2))])
def test_dd_processes_gloo(tmp_path, m, n, P, Ld, grid):
    """Ranks in separate processes (TorchComm over gloo: device halos staged through the host, column
    strips packed), the path the RCCL run takes with device buffers; slabs and 2-D blocks."""
    mp.spawn(_dd_worker, args=(P, m, n, Ld, _free_port(), str(tmp_path), grid), nprocs=P, join=True)
    got = np.full((1, 1, m + 1, n + 1), np.nan)
    for r in range(P):
        y0, y1, x0, x1 = np.load(os.path.join(tmp_path, f"i{r}.npy"))
        got[:, :, y0:y1, x0:x1] = np.load(os.path.join(tmp_path, f"r{r}.npy"))
    f, u0, bc = _global_problem(m, n, 1)
    _, ref = _single(m, n, 1, f, u0, bc, 3)
    exp = ref[-1][0].cpu().numpy()
    assert np.array_equal(got, exp), np.nanmax(np.abs(got - exp))
    for r in range(P):
        np.testing.assert_allclose(np.load(os.path.join(tmp_path, f"n{r}.npy")), ref[-1][1].cpu().numpy(), rtol=1e-12)
