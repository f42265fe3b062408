"""GPU parity of the decomposed periodic Jacobi sweeps (feanet_amd/pbc_dd.py, HIP local sweeps +
periodic halo exchange): P processes on the one GPU exchanging over gloo, gathered result BITWISE the
single-GPU periodic sweep fea_jacobi_sweep_pbc applied the same number of times (same per-node expression
and summation order), fp64 and fp32, row slabs and 2 x 2 blocks, 1 and 3 ghost lines per exchange.
(The oracle is imported only to build the periodic test input.)"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SWEEPS = 7


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(n, B, T):
    """Random iterate and a PERIODIC forcing term (the circular extension of a random field, as the
    reference's drivers build it: FNet of the periodic extension): then the last row / column of a sweep
    equal the first, which is how the decomposed sweep assembles them."""
    from oracle import feanet_oracle as orc
    g = torch.Generator().manual_seed(n + B)
    u = torch.randn(B, 1, n + 1, n + 1, generator=g, dtype=torch.float64).to(T)
    F = torch.randn(B, 1, n + 1, n + 1, generator=g, dtype=torch.float64)
    f = torch.from_numpy(orc.pbc_pad(F.numpy(), 1, 2)).to(T)
    return u, f


def _tables(T):
    from feanet_amd import mesh_setup as ms
    ktab3 = ms.stencil_table(None)
    return ktab3, ms.omega_over_d(ktab3, 2. / 3., np.float32 if T == torch.float32 else np.float64)


def _run(rank, world, grid, G, n, B, tname, port, outdir):
    import torch.distributed as dist
    from feanet_amd.pbc_dd import PeriodicComm, PeriodicJacobiDD
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    T = getattr(torch, tname)
    u, f = _problem(n, B, T)
    ktab3, omd = _tables(T)
    s = PeriodicJacobiDD(n, rank, grid, ktab3[0], omd, comm=PeriodicComm(), ghost=G, batch=B, dtype=T)
    s.set_rhs(f.cuda())
    s.load(u.cuda())
    s.sweep(SWEEPS)
    out = s.gather()
    torch.cuda.synchronize()
    if rank == 0:
        torch.save(out.cpu(), os.path.join(outdir, "out.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("grid,G,n,B,tname", [((2, 1), 1, 64, 2, "float64"), ((2, 2), 3, 64, 1, "float64"),
                                              ((1, 2), 3, 256, 2, "float32"), ((2, 2), 1, 130, 1, "float32")])
def test_periodic_dd_bitwise_single_gpu(tmp_path, grid, G, n, B, tname):
    from feanet_amd import ops
    world = grid[0] * grid[1]
    mp.spawn(_run, args=(world, grid, G, n, B, tname, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = torch.load(os.path.join(tmp_path, "out.pt"), weights_only=True)
    T = getattr(torch, tname)
    u, f = _problem(n, B, T)
    ktab3, omd = _tables(T)
    v, fc = u.cuda(), f.cuda()
    for _ in range(SWEEPS):
        v = ops.jacobi_sweep_pbc(v, fc, torch.from_numpy(ktab3), omd)
    assert torch.equal(got, v.cpu()), (got - v.cpu()).abs().max().item()


def test_periodic_dd_single_rank_hip():
    """One rank (its own neighbour along both axes: local copies only), HIP sweeps, bitwise."""
    from feanet_amd import ops
    from feanet_amd.pbc_dd import PeriodicJacobiDD
    n, B, T = 96, 2, torch.float64
    u, f = _problem(n, B, T)
    ktab3, omd = _tables(T)
    s = PeriodicJacobiDD(n, 0, (1, 1), ktab3[0], omd, ghost=2, batch=B, dtype=T)
    s.set_rhs(f.cuda())
    s.load(u.cuda())
    s.sweep(5)
    v, fc = u.cuda(), f.cuda()
    for _ in range(5):
        v = ops.jacobi_sweep_pbc(v, fc, torch.from_numpy(ktab3), omd)
    assert torch.equal(s.gather(), v)
