"""Periodic Jacobi sweeps on a domain-decomposed grid (feanet_amd/pbc_dd.py; SURVEY §8f row 4, the periodic
halo exchange of the multi-GPU case) over gloo, world sizes 1..4, row slabs, column slabs and 2 x 2 blocks,
1 and 2 ghost lines per exchange.  The local sweep is the oracle's generic Jacobi sweep (reset mask one,
zero boundary values: the semantics of the HIP kernel the product path runs, fea_jacobi_sweep); the
gathered result is pinned by the reference's OWN periodic outputs (tests/golden/pbc_jacobi.npz: one and
three sweeps of JacobiBlockPBC.jacobi_convolution, FEANet/jacobi.py:86-97, and 30 sweeps of the periodic
single-grid driver of FEANet-periodic.ipynb from zero), fp64 to 1e-13 and fp32 to 1e-5 of max(1, max|u|).
The GPU test (tests/test_gpu_pbc_dd.py) checks the HIP path bitwise against fea_jacobi_sweep_pbc."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import feanet_oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_sweep(ktab, dt):
    def sweep(u, f, out):
        un, fn = u.numpy(), f.numpy()
        H, W = un.shape[-2:]
        res = orc.jacobi_sweep(un, fn, np.zeros((H, W), np.uint8), ktab, np.ones((H, W), dt), dt(0))
        out.copy_(torch.from_numpy(np.ascontiguousarray(res)))
    return sweep


def _run(rank, world, grid, G, tag, n, port, outdir):
    import torch.distributed as dist
    from feanet_amd import mesh_setup as ms
    from feanet_amd.pbc_dd import PeriodicComm, PeriodicJacobiDD
    if world > 1:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dt = np.float32 if tag == "f32" else np.float64
    g = np.load(os.path.join(HERE, "golden", "pbc_jacobi.npz"))
    ktab3 = ms.stencil_table(None)  # [1, 3, 3]
    ktab = ktab3[0]
    omd = ms.omega_over_d(ktab3, 2. / 3., dt)
    T = torch.float32 if tag == "f32" else torch.float64
    u, f = g[f"{tag}_n{n}_u"], g[f"{tag}_n{n}_f"]
    B = u.shape[0]
    s = PeriodicJacobiDD(n, rank, grid, ktab, omd, comm=PeriodicComm() if world > 1 else None, ghost=G, batch=B,
                         dtype=T, device="cpu", local_sweep=_oracle_sweep(ktab3, dt))
    s.set_rhs(torch.from_numpy(f))
    s.load(torch.from_numpy(u))
    s.sweep(1)
    u1 = s.gather().numpy()
    s.sweep(2)
    u3 = s.gather().numpy()
    s.set_rhs(torch.from_numpy(f[:1]).expand(B, -1, -1, -1))
    s.load(None)
    s.sweep(30)
    v30 = s.gather().numpy()
    if rank == 0:
        np.savez(os.path.join(outdir, "out.npz"), u1=u1, u3=u3, v30=v30[:1])
    if world > 1:
        dist.destroy_process_group()


@pytest.mark.parametrize("grid,G,tag,n", [((1, 1), 1, "f64", 16), ((2, 1), 1, "f64", 16), ((1, 2), 2, "f64", 16),
                                          ((2, 2), 1, "f64", 16), ((2, 2), 2, "f64", 32), ((3, 1), 2, "f64", 32),
                                          ((1, 4), 1, "f64", 8), ((2, 1), 2, "f32", 8), ((2, 2), 1, "f32", 16),
                                          ((1, 3), 1, "f32", 32)])
def test_periodic_dd_matches_reference(tmp_path, grid, G, tag, n):
    world = grid[0] * grid[1]
    if n < max(grid) * G:
        pytest.skip("blocks thinner than the ghost depth")
    if world == 1:
        _run(0, 1, grid, G, tag, n, 0, str(tmp_path))
    else:
        mp.spawn(_run, args=(world, grid, G, tag, n, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = np.load(os.path.join(tmp_path, "out.npz"))
    gold = np.load(os.path.join(HERE, "golden", "pbc_jacobi.npz"))
    tol = 1e-5 if tag == "f32" else 1e-13
    for k in ("u1", "u3", "v30"):
        ref = gold[f"{tag}_n{n}_{k}"]
        err = np.abs(got[k] - ref).max() / max(1.0, np.abs(ref).max())
        assert err <= tol, (k, err)


def test_periodic_dd_rejects_thin_blocks():
    from feanet_amd.pbc_dd import PeriodicJacobiDD
    with pytest.raises(ValueError):
        PeriodicJacobiDD(8, 0, (4, 1), np.ones(9), [1.0], ghost=3, device="cpu")
    with pytest.raises(ValueError):
        PeriodicJacobiDD(8, 4, (2, 2), np.ones(9), [1.0], device="cpu")
