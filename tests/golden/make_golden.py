#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by RUNNING the reference
(longfish/Multigrid-FEANet, read-only at /root/reference) on the CPU of the build
container.  Only this script touches the reference; the fixtures it writes are
plain data (inputs + expected outputs, .npz, allow_pickle=False) and are what the
test-suite, the oracle pinning and the GPU parity tests read.  Nothing of the
reference's source travels with the fixtures.

How the reference is run (SURVEY.md §8c recipe):
  * `meshio` is not installed; the reference uses it only as a container for
    points/cells/cell_data (FEANet/mesh.py:60,68,169) and for VTK export, which
    is never called here.  A tiny in-memory container is registered under that
    module name for the duration of this script.
  * `h5py` is not installed; every dataset used is a contiguous little-endian
    float64 block, read with np.fromfile at the offsets listed in SURVEY §8c.
  * Notebook classes (MultiGrid.Step, Multigrid.rec_V_cycle, ...) are executed
    from the code cells of the notebooks' JSON.
  * FEANet/multigrid.py:46 passes n_iter= to jacobi_convolution, which raises
    TypeError; SingleGrid.Relax is patched to loop single sweeps,
    the intended semantics.

Usage:  python tests/golden/make_golden.py   (≈1 min)
"""
import json
import os
import sys
import time
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# reference import harness
# --------------------------------------------------------------------------
def _install_meshio_container():
    mod = types.ModuleType("meshio")

    class Mesh:  # points/cells holder only; no I/O
        def __init__(self, points, cells):
            self.points = points
            self.cells = cells
            self.cell_data = {}

        def write(self, *a, **k):
            raise RuntimeError("VTK export is not available in the fixture harness")

    mod.Mesh = Mesh
    sys.modules["meshio"] = mod


_install_meshio_container()
sys.path.insert(0, REF)

import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from functools import reduce  # noqa: E402
import math  # noqa: E402
import random  # noqa: E402

from FEANet.geo import Geometry  # noqa: E402
from FEANet.jacobi import JacobiBlock  # noqa: E402
from FEANet.mesh import MeshCenterInterface, MeshSquare  # noqa: E402
from FEANet.model import FNet, KNet  # noqa: E402
import FEANet.multigrid as ref_mg  # noqa: E402


def _patched_relax(self, v, f, num_sweeps_down):
    for _ in range(num_sweeps_down):
        v = self.jac.jacobi_convolution(v, f)
    return v


ref_mg.SingleGrid.Relax = _patched_relax


def nb_cells(path, idx):
    d = json.load(open(os.path.join(REF, path)))
    return ["".join(d["cells"][i]["source"]) for i in idx]


def nb_namespace(path, idx, extra=None):
    ns = dict(torch=torch, nn=nn, F=F, np=np, math=math, random=random, time=time,
              os=os, reduce=reduce, Geometry=Geometry, JacobiBlock=JacobiBlock,
              MeshSquare=MeshSquare, MeshCenterInterface=MeshCenterInterface,
              KNet=KNet, FNet=FNet, DataLoader=None)
    if extra:
        ns.update(extra)
    for src in nb_cells(path, idx):
        exec(compile(src, f"{path}", "exec"), ns)
    return ns


def seed(s):
    np.random.seed(s)
    random.seed(s)
    torch.manual_seed(s)


def pid_from_global_pattern(mesh):
    n = mesh.nnode_edge
    keys = sorted(mesh.kernel_dict)
    stack = np.stack([mesh.global_pattern_center[k].reshape(n, n) for k in keys])
    assert (stack.sum(0) == 1).all(), "every node must carry exactly one pattern"
    return np.argmax(stack, axis=0).astype(np.uint8)


def kernels(mesh):
    return np.stack([mesh.kernel_dict[k] for k in sorted(mesh.kernel_dict)]).astype(np.float32)


def t2n(t):
    return t.detach().cpu().numpy().copy()  # never alias a tensor the reference mutates in place (Q6)


def save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **arrays)
    print("wrote", name, sorted(arrays))


# --------------------------------------------------------------------------
# dataset readers (contiguous float64, SURVEY §8c offsets)
# --------------------------------------------------------------------------
def read_block(path, offset, shape):
    cnt = int(np.prod(shape))
    return np.fromfile(os.path.join(REF, path), dtype="<f8", count=cnt, offset=offset).reshape(shape)


def iso_poisson_33(nsamp):
    p = "Data/IsoPoisson/poisson2d_33x33.h5"
    shp = (100, 33, 33)
    return {k: read_block(p, off, shp)[:nsamp] for k, off in
            [("boundary_index", 2048), ("boundary_value", 873248), ("rhs", 1744448), ("u", 2617696)]}


def test_poisson_33(nsamp):
    p = "Data/TestPoisson/poisson2d_33x33.h5"
    out = {}
    for k, off, shp in [("dirich_idx", 2048, (10, 33, 33)), ("dirich_value", 89168, (10, 33, 33)),
                        ("material", 352576, (10, 32, 32, 1)), ("source", 434496, (10, 33, 33)),
                        ("solution", 521616, (10, 33, 33))]:
        out[k] = read_block(p, off, shp)[:nsamp]
    return out


# --------------------------------------------------------------------------
# 1. setup tables: stencils, pattern maps, mass stencils, masks
# --------------------------------------------------------------------------
def gen_tables():
    arr = {}
    arr["square_kernel"] = kernels(MeshSquare(2, 9))
    for shape in (0, 1):
        for n in (5, 9, 17, 33, 65, 129):
            m = MeshCenterInterface(2, [1, 20], n, shape)
            arr[f"iface{shape}_pid_{n}"] = pid_from_global_pattern(m)
            arr[f"iface{shape}_kernel_{n}"] = kernels(m)
    m = MeshCenterInterface(2, [3, 7], 17, 0)
    arr["iface0_prop3_7_kernel"] = kernels(m)
    for n in (2, 4, 16, 32, 64, 128, 4096):
        arr[f"fnet_{n}"] = t2n(FNet(2 / n).net.weight)[0, 0]
    g = Geometry(17)
    arr["geo_17"] = t2n(g.geometry_idx)
    arr["bc_17"] = t2n(g.boundary_value)
    save("tables.npz", **arr)


# --------------------------------------------------------------------------
# 2. single-op I/O (KNet, split_x, FNet, Jacobi, residual, R, P)
# --------------------------------------------------------------------------
def gen_ops():
    mg_ns = nb_namespace("M-FEANet-mg_test.ipynb", [18])  # 1-channel R/P nets
    mm_ns = nb_namespace("MM_Model_convergence.ipynb", [2, 3])
    lin = torch.asarray([[1, 2, 1], [2, 4, 2], [1, 2, 1]], dtype=torch.float32)
    sd = torch.load(os.path.join(REF, "Model/learn_intergrid_operator/multigrid_rhs_qm/"
                                      "model_multigrid_interface_ratio.pth"), weights_only=True)
    for dt in ("f32", "f64"):
        torch.set_default_dtype(torch.float64 if dt == "f64" else torch.float32)
        tdt = torch.get_default_dtype()
        for case in ("poisson", "iface0", "iface1"):
            for n in (16, 32):
                N = n + 1
                seed(1000 + n)
                mesh = MeshSquare(2, N) if case == "poisson" else \
                    MeshCenterInterface(2, [1, 20], N, 0 if case == "iface0" else 1)
                knet = KNet(mesh)
                fnet = FNet(2 / n)
                if dt == "f64":
                    knet = knet.double()
                    fnet = fnet.double()
                geo = Geometry(N)
                bc = geo.boundary_value.clone()
                edge = torch.rand(4, dtype=tdt)
                bc[0, 0, -1, :] = edge[0]
                bc[0, 0, 0, :] = edge[1]
                bc[0, 0, :, -1] = edge[2]
                bc[0, 0, :, 0] = edge[3]
                jac = JacobiBlock(knet, mesh, 2 / 3., geo.geometry_idx, bc)
                B = 2
                u = torch.randn(B, 1, N, N, dtype=tdt)
                f = torch.randn(B, 1, N, N, dtype=tdt)
                Fsrc = torch.randn(B, 1, N, N, dtype=tdt)
                e_c = torch.randn(B, 1, n // 2 + 1, n // 2 + 1, dtype=tdt)
                e_c[:, :, 0, :] = 0
                e_c[:, :, -1, :] = 0
                e_c[:, :, :, 0] = 0
                e_c[:, :, :, -1] = 0
                with torch.no_grad():
                    out = dict(u=t2n(u), f=t2n(f), F=t2n(Fsrc), e_c=t2n(e_c),
                               pid=pid_from_global_pattern(mesh) if case != "poisson" else np.zeros((N, N), np.uint8),
                               ktab=kernels(mesh), geo=t2n(geo.geometry_idx), bc=t2n(bc),
                               d_mat=t2n(jac.d_mat))
                    out["knet"] = t2n(knet(u))
                    out["split"] = t2n(knet.split_x(u))
                    out["fnet"] = t2n(fnet(Fsrc))
                    out["jacobi"] = t2n(jac.jacobi_convolution(u, f))
                    out["jacobi2"] = t2n(jac.jacobi_convolution(jac.jacobi_convolution(u, f), f))
                    out["residual"] = t2n(f - knet(u))
                    if case == "poisson":
                        Rn = mg_ns["RestrictionNet"](lin / 4.0)
                        Pn = mg_ns["ProlongationNet"](lin / 4.0)
                        if dt == "f64":
                            Rn, Pn = Rn.double(), Pn.double()
                        r = f - knet(u)
                        rc = Rn(knet.split_x(r)[:, :, 1:-1, 1:-1])
                        out["restrict_mgtest"] = t2n(F.pad(rc, (1, 1, 1, 1), "constant", 0))
                        out["prolong_mgtest"] = t2n(Pn(e_c))
                        if dt == "f32":  # the MM notebooks hard-code a float32 kernel (fp64 raises there)
                            mm = mm_ns["Multigrid"](n)
                            out["restrict_mm"] = t2n(4 * mm.Restrict(r))
                            out["interp_mm"] = t2n(mm.Interpolate(e_c))
                    else:
                        mgm = ref_mg.MultiGrid(n, lin / 16.0, lin / 4.0, torch.tensor([4.0, 1.0]))
                        mgm.load_state_dict(sd)
                        if dt == "f64":
                            mgm = mgm.double()
                        r = f - knet(u)
                        w = mgm.w.detach()
                        out["w"] = t2n(w)
                        out["rtab"] = t2n(mgm.conv.net.weight)[0].reshape(16, 3, 3)
                        out["ptab"] = t2n(mgm.deconv.net.weight)[:, 0].reshape(16, 3, 3)
                        coarse_mesh = mgm.grids[1].grid
                        out["pid_c"] = pid_from_global_pattern(coarse_mesh)
                        out["restrict_learned"] = t2n(w[0] * mgm.Restrict(mgm.grids[0].Knet.split_x(r)))
                        out["prolong_learned"] = t2n(w[1] * mgm.Interpolate(mgm.grids[1].Knet.split_x(e_c)))
                save(f"ops_{case}_{dt}_n{n}.npz", **out)
    torch.set_default_dtype(torch.float32)


# --------------------------------------------------------------------------
# 3. V-cycle histories
# --------------------------------------------------------------------------
def mg_test_runs():
    """M-FEANet-mg_test.ipynb MultiGrid.Step (cells 19, 21, 22) on IsoPoisson 33²."""
    ns = nb_namespace("M-FEANet-mg_test.ipynb", [2, 3, 4, 5, 18, 19, 20])
    hnet = ns["HNet"](3)
    hnet.load_state_dict(torch.load(os.path.join(REF, "Model/learn_iterator/iso_poisson/iso_poisson_33x33.pth"),
                                    weights_only=True))
    data = iso_poisson_33(5)
    n = 32
    out = {k: v for k, v in data.items()}
    out["hnet_w"] = np.stack([t2n(hnet.convLayers[i].weight)[0, 0] for i in range(3)])
    P = ns["linear_tensor_P"]
    for mode in ("jac", "hjac"):
        for k in range(3):
            seed(0)
            mg = ns["MultiGrid"](n=n, hnet=hnet, P=P, mode=mode)
            mg.requires_grad_(False)
            f_mg = torch.from_numpy(data["rhs"][k].astype(np.float32)).reshape(1, 1, n + 1, n + 1)
            bci = torch.from_numpy(data["boundary_index"][k].astype(np.float32)).reshape(1, 1, n + 1, n + 1)
            bcv = torch.from_numpy(data["boundary_value"][k].astype(np.float32)).reshape(1, 1, n + 1, n + 1)
            u_mg = torch.zeros((1, 1, n + 1, n + 1), dtype=torch.float32)
            with torch.no_grad():
                mg(u_mg, f_mg, bci, bcv, 1)
                residual = mg.f - mg.iterators[0].grid.Knet(mg.u0)
                res = torch.norm(residual[:, :, 1:-1, 1:-1].clone(), dim=(2, 3)).item()
                hist = [res]
                first = None
                while abs(res) > 5e-5 and len(hist) < 60:
                    u_mg = mg.Step(u_mg, mg.f)
                    if first is None:
                        first = t2n(u_mg)
                    residual = mg.f - mg.iterators[0].grid.Knet(u_mg)
                    res = torch.norm(residual[:, :, 1:-1, 1:-1].clone(), dim=(2, 3)).item()
                    hist.append(res)
            out[f"{mode}_hist_{k}"] = np.array(hist)
            out[f"{mode}_u_final_{k}"] = t2n(u_mg)
            out[f"{mode}_u_first_{k}"] = first
            out[f"{mode}_fnet_f_{k}"] = t2n(mg.f)
            print(f"mg_test {mode} sample {k}: {len(hist) - 1} cycles, final {hist[-1]:.3e}")
    # one HRelax sweep on random input (HNet smoother, row (f) of the scope table)
    seed(7)
    it = ns["HJacIterator"](n=n, hnet=hnet)
    u = torch.randn(2, 1, n + 1, n + 1)
    f = torch.randn(2, 1, n + 1, n + 1)
    with torch.no_grad():
        out["hrelax_u"] = t2n(u)
        out["hrelax_f"] = t2n(f)
        out["hrelax_out1"] = t2n(it.HRelax(u, f, 1))
        out["hrelax_out3"] = t2n(it.HRelax(u, f, 3))
    save("mg_test_isopoisson33.npz", **out)


def mg_test_synthetic():
    """mg_test Step on synthetic 65² problems: L=6 and L=3 (BASELINE config 1), fp32 and fp64."""
    gr_ns = {}
    exec(open(os.path.join(REF, "Data/RHS/gaussian_random_fields.py")).read(), gr_ns)
    out = {}
    for dt in ("f32", "f64"):
        torch.set_default_dtype(torch.float64 if dt == "f64" else torch.float32)
        ns = nb_namespace("M-FEANet-mg_test.ipynb", [2, 3, 4, 5, 18, 19, 20])
        hnet = ns["HNet"](3)
        n = 64
        N = n + 1
        seed(42)
        alpha = random.uniform(5, 10)
        a = random.uniform(1, 5)
        Fsrc = a * gr_ns["gaussian_random_field"](alpha=alpha, size=N)
        bcvals = np.random.rand(4)
        geo = np.ones((N, N))
        geo[0, :] = geo[-1, :] = geo[:, 0] = geo[:, -1] = 0
        bcv = np.zeros((N, N))
        bcv[-1, :] = bcvals[0]
        bcv[0, :] = bcvals[1]
        bcv[:, -1] = bcvals[2]
        bcv[:, 0] = bcvals[3]
        tdt = torch.get_default_dtype()
        f_mg = torch.tensor(Fsrc, dtype=tdt).reshape(1, 1, N, N)
        bci = torch.tensor(geo, dtype=tdt).reshape(1, 1, N, N)
        bcvt = torch.tensor(bcv, dtype=tdt).reshape(1, 1, N, N)
        out[f"{dt}_F"] = Fsrc
        out[f"{dt}_geo"] = geo
        out[f"{dt}_bc"] = bcv
        for L in (6, 3):
            mg = ns["MultiGrid"](n=n, hnet=hnet, P=ns["linear_tensor_P"], mode="jac")
            mg.requires_grad_(False)
            if dt == "f64":
                for i in mg.iterators:
                    mg.iterators[i].grid.fnet = mg.iterators[i].grid.fnet.double()
            mg.L = L
            u_mg = torch.zeros((1, 1, N, N), dtype=torch.float32)
            with torch.no_grad():
                mg(u_mg, f_mg, bci, bcvt, 1)
                residual = mg.f - mg.iterators[0].grid.Knet(mg.u0)
                res = torch.norm(residual[:, :, 1:-1, 1:-1].clone(), dim=(2, 3)).item()
                hist = [res]
                eps = 1e-9 if dt == "f64" else 5e-6
                while abs(res) > eps and len(hist) < (40 if L == 6 else 25):
                    u_mg = mg.Step(u_mg, mg.f)
                    residual = mg.f - mg.iterators[0].grid.Knet(u_mg)
                    res = torch.norm(residual[:, :, 1:-1, 1:-1].clone(), dim=(2, 3)).item()
                    hist.append(res)
            out[f"{dt}_L{L}_hist"] = np.array(hist)
            out[f"{dt}_L{L}_u_final"] = t2n(u_mg)
            out[f"{dt}_fnet_f"] = t2n(mg.f)
            print(f"mg_test synthetic {dt} L={L}: {len(hist) - 1} cycles, final {hist[-1]:.3e}")
    torch.set_default_dtype(torch.float32)
    save("mg_test_synth65.npz", **out)


def mm_convergence_runs():
    """MM_Model_convergence.ipynb Multigrid.Solve / rec_V_cycle (cells 2, 3): V(nu1,nu2) histories."""
    ns = nb_namespace("MM_Model_convergence.ipynb", [2, 3])

    def random_data_numpy1(self):
        # Multigrid.random_data (MM_Model_convergence.ipynb cell 3) relies on NumPy-1 value-based
        # casting (float64 scalar * float32 array -> float32); NumPy 2 promotes to float64 and the
        # fp32 KNet then raises.  Same draws, NumPy-1 arithmetic.
        coef = 100000 + 50000 * np.random.rand(2)
        a = np.random.random((self.n + 1, self.n + 1)).astype("f")
        return np.float32(coef[0]) * a + np.float32(coef[1])

    ns["Multigrid"].random_data = random_data_numpy1
    out = {}
    for n in (16, 32, 64):
        for nu in ((1, 1), (0, 1), (1, 0), (2, 1), (1, 2), (2, 2), (0, 2), (2, 0)):
            seed(n * 10 + nu[0] * 3 + nu[1])
            mg = ns["Multigrid"](n)
            out[f"n{n}_v{nu[0]}{nu[1]}_init"] = t2n(mg.initial_v)
            with torch.no_grad():
                hist = mg.Solve(list(nu), rec=True, n_iter=10)
            out[f"n{n}_v{nu[0]}{nu[1]}_hist"] = np.array(hist)
            out[f"n{n}_v{nu[0]}{nu[1]}_u"] = t2n(mg.grids[0].v)
        seed(n)
        mg = ns["Multigrid"](n, final_level=3)
        out[f"n{n}_L3_init"] = t2n(mg.initial_v)
        with torch.no_grad():
            out[f"n{n}_L3_hist"] = np.array(mg.Solve([1, 1], rec=True, n_iter=10))
        seed(n + 1)
        mg = ns["Multigrid"](n)
        out[f"n{n}_jac_init"] = t2n(mg.initial_v)
        with torch.no_grad():
            out[f"n{n}_jac_hist"] = np.array(mg.solve_jacobi(n_iter=30))
    save("mm_convergence.npz", **out)


def mm_interface_run():
    """MM_Interface_error.ipynb (cells 1, 2, 13, 14): two-material 65², f = FNet(1), u0 = 0,
    V-cycle with the notebook's grids[0] pre-smoothing, EPS 5e-5."""
    ns = nb_namespace("MM_Interface_error.ipynb", [1, 2])
    n = 64
    mg = ns["Multigrid"](n)
    mg.grids[0].v = torch.zeros((1, 1, n + 1, n + 1), dtype=torch.float32)
    res = 1
    hist = []
    err = []
    with torch.no_grad():
        while abs(res) > 5e-5 and len(hist) < 40:
            u_prev = mg.grids[0].v
            mg.rec_V_cycle(0, mg.grids[0].v, mg.grids[0].f)
            e = torch.sqrt(torch.sum((mg.grids[0].v - u_prev) ** 2)).item() / \
                torch.sqrt(torch.sum(mg.grids[0].v ** 2)).item()
            residual = mg.grids[0].f - mg.grids[0].Knet(mg.grids[0].v)
            res = torch.sqrt(torch.sum(residual[:, :, 1:-1, 1:-1] ** 2)).item()
            hist.append(res)
            err.append(e)
    print(f"MM_Interface 65²: {len(hist)} cycles, final {hist[-1]:.3e}")
    save("mm_interface65.npz", hist=np.array(hist), rel_change=np.array(err), u_final=t2n(mg.grids[0].v),
         f=t2n(mg.grids[0].f))


def multigrid_py_runs():
    """FEANet/multigrid.py MultiGrid.iterate (two-material, 16-channel learned R/P, w) at 65²."""
    lin = torch.asarray([[1, 2, 1], [2, 4, 2], [1, 2, 1]], dtype=torch.float32)
    sd = torch.load(os.path.join(REF, "Model/learn_intergrid_operator/multigrid_rhs_qm/"
                                      "model_multigrid_interface_ratio.pth"), weights_only=True)
    out = {}
    n = 64
    for tag in ("linear", "learned"):
        mg = ref_mg.MultiGrid(n, lin / 16.0, lin / 4.0, torch.tensor([4.0, 1.0]))
        if tag == "learned":
            mg.load_state_dict(sd)
        with torch.no_grad():
            F1 = torch.ones(1, 1, n + 1, n + 1)
            f = mg.grids[0].fnet(F1)
            u = torch.zeros(1, 1, n + 1, n + 1)
            r = f - mg.grids[0].Knet(u)
            hist = [torch.norm(r[:, :, 1:-1, 1:-1], dim=(2, 3)).item()]
            while hist[-1] > 5e-5 and len(hist) < 40:
                u = mg.iterate(u, f)
                r = f - mg.grids[0].Knet(u)
                hist.append(torch.norm(r[:, :, 1:-1, 1:-1], dim=(2, 3)).item())
        out[f"{tag}_hist"] = np.array(hist)
        out[f"{tag}_u"] = t2n(u)
        out[f"{tag}_w"] = t2n(mg.w)
        out[f"{tag}_rtab"] = t2n(mg.conv.net.weight)[0].reshape(16, 3, 3)
        out[f"{tag}_ptab"] = t2n(mg.deconv.net.weight)[:, 0].reshape(16, 3, 3)
        print(f"multigrid.py {tag}: {len(hist) - 1} cycles, final {hist[-1]:.3e}")
    out["f"] = t2n(f)
    for l in range(int(np.log2(n))):
        out[f"pid_level{l}"] = pid_from_global_pattern(mg.grids[l].grid)
    save("multigrid_py_iface65.npz", **out)


def multigrid_py_training():
    """FEANet/multigrid.py training forward (MultiGrid.forward + qm, :132-157) and its backward:
    the gradients of q_m w.r.t. the 16-channel restriction / prolongation kernels (§8f row 2).
    np.random is seeded right before forward(), which draws the random initial guesses."""
    lin = torch.asarray([[1, 2, 1], [2, 4, 2], [1, 2, 1]], dtype=torch.float32)
    sd = torch.load(os.path.join(REF, "Model/learn_intergrid_operator/multigrid_rhs_qm/"
                                      "model_multigrid_interface_ratio.pth"), weights_only=True)
    out = {}
    for n, B, tag in ((16, 2, "linear"), (32, 2, "learned")):
        mg = ref_mg.MultiGrid(n, lin / 16.0, lin / 4.0, torch.tensor([4.0, 1.0]))
        if tag == "learned":
            mg.load_state_dict(sd)
        seed(100 + n)
        F1 = torch.from_numpy(np.random.default_rng(n).random((B, 1, n + 1, n + 1)).astype(np.float32))
        np.random.seed(1000 + n)
        u = mg(F1)
        loss = mg.qm(u)
        loss.backward()
        k = f"n{n}_"
        out[k + "F"] = t2n(F1)
        out[k + "v0"] = t2n(mg.v)
        out[k + "u"] = t2n(u)
        out[k + "loss"] = np.array(loss.item())
        out[k + "rtab"] = t2n(mg.conv.net.weight)[0]
        out[k + "ptab"] = t2n(mg.deconv.net.weight)[:, 0]
        out[k + "w"] = t2n(mg.w)
        out[k + "grad_R"] = t2n(mg.conv.net.weight.grad)[0]
        out[k + "grad_P"] = t2n(mg.deconv.net.weight.grad)[:, 0]
        print(f"multigrid.py training n={n}: q_m={loss.item():.6f}")
    save("multigrid_py_training.npz", **out)


def recorded_outputs():
    """Known answers the reference's notebooks hold in their stored outputs."""
    import re
    out = {}
    d = json.load(open(os.path.join(REF, "MM_Interface_error.ipynb")))
    txt = "".join(d["cells"][14]["outputs"][0]["text"])
    rows = [l.split() for l in txt.splitlines() if re.match(r"^[0-9.e+-]+ [0-9.e+-]+$", l.strip())]
    out["mm_interface_rel_change"] = np.array([float(r[0]) for r in rows])
    out["mm_interface_res"] = np.array([float(r[1]) for r in rows])
    d = json.load(open(os.path.join(REF, "MM_Model_convergence.ipynb")))
    txt = "".join(d["cells"][5]["outputs"][0]["text"])
    out["mm_vcycle_q_by_log2n"] = np.array([float(x) for x in re.findall(r"is: ([0-9.]+)", txt)])
    txt = "".join(d["cells"][6]["outputs"][0]["text"])
    out["mm_jacobi_q_by_log2n"] = np.array([float(x) for x in re.findall(r"is: ([0-9.]+)", txt)])
    q = []
    for c in (9, 10, 11, 12, 13, 14, 15, 16):
        txt = "".join("".join(o.get("text", "")) for o in d["cells"][c]["outputs"])
        q.append(float(re.findall(r"factor is: ([0-9.]+)", txt)[0]))
    out["mm_vnu_q_n64"] = np.array(q)  # V(0,1) V(0,2) V(1,0) V(1,1) V(1,2) V(2,0) V(2,1) V(2,2)
    save("recorded_outputs.npz", **out)
    print({k: v[:4] for k, v in out.items()})


def dataset_fixtures():
    d = iso_poisson_33(5)
    t = test_poisson_33(2)
    save("datasets.npz", **{f"iso_{k}": v for k, v in d.items()}, **{f"test_{k}": v for k, v in t.items()})


def weights():
    """Learned operators shipped with the reference (Model/), copied as plain arrays: the inputs of
    BASELINE config 3 (learned R/P ratio) and of the HNet smoother."""
    wdir = os.path.join(os.path.dirname(OUT), "..", "multigrid-feanet_amd", "feanet_amd", "weights")
    sd = torch.load(os.path.join(REF, "Model/learn_intergrid_operator/multigrid_rhs_qm/"
                                      "model_multigrid_interface_ratio.pth"), weights_only=True)
    np.savez(os.path.join(wdir, "multigrid_interface_ratio.npz"),
             w=sd["w"].numpy(), R=sd["conv.net.weight"].numpy(), P=sd["deconv.net.weight"].numpy())
    sd = torch.load(os.path.join(REF, "Model/learn_iterator/iso_poisson/iso_poisson_33x33.pth"), weights_only=True)
    np.savez(os.path.join(wdir, "hnet_iso_poisson_33x33.npz"),
             **{f"conv{i}": sd[f"convLayers.{i}.weight"].numpy() for i in range(3)})
    print("wrote weights")


def pbc_runs():
    """JacobiBlockPBC (FEANet/jacobi.py:50-97) on MeshSquare grids: circular extension, reset, one and
    three periodic sweeps, and the residual history of the periodic single-grid driver of
    Archive/FEA-Net/MM-FEANet/FEANet-periodic.ipynb (cells 2, 5: f = FNet(pbc_boundary(F)),
    res = ||(f - K pbc_boundary(u))[1:-1, 1:-1]||), in fp32 and fp64."""
    from FEANet.jacobi import JacobiBlockPBC
    out = {}
    for tag, dt in (("f32", torch.float32), ("f64", torch.float64)):
        torch.set_default_dtype(dt)
        for n in (8, 16, 32):
            N = n + 1
            seed(100 + n)
            mesh = MeshSquare(2.0, nnode_edge=N)
            knet = KNet(mesh)
            fnet = FNet(2.0 / n)
            if dt == torch.float64:
                knet, fnet = knet.double(), fnet.double()
            jac = JacobiBlockPBC(mesh, knet, 2. / 3.)
            B = 2
            u = torch.randn(B, 1, N, N, dtype=dt)
            Fs = torch.randn(B, 1, N, N, dtype=dt)
            with torch.no_grad():
                f = fnet(jac.pbc_boundary(Fs))
                u1 = jac.jacobi_convolution(u, f)
                u3 = u1
                for _ in range(2):
                    u3 = jac.jacobi_convolution(u3, f)
                v = torch.zeros(1, 1, N, N, dtype=dt)
                hist = []
                f0 = f[:1]
                for _ in range(30):
                    v = jac.jacobi_convolution(v, f0)
                    r = f0 - knet(jac.pbc_boundary(v))
                    hist.append(torch.sqrt(torch.sum(r[:, :, 1:-1, 1:-1] ** 2)).item())
                out.update({f"{tag}_n{n}_u": t2n(u), f"{tag}_n{n}_F": t2n(Fs), f"{tag}_n{n}_f": t2n(f),
                            f"{tag}_n{n}_pbc": t2n(jac.pbc_boundary(u)), f"{tag}_n{n}_reset": t2n(jac.reset_boundary(u)),
                            f"{tag}_n{n}_u1": t2n(u1), f"{tag}_n{n}_u3": t2n(u3), f"{tag}_n{n}_hist": np.array(hist),
                            f"{tag}_n{n}_v30": t2n(v), f"{tag}_n{n}_dmat": t2n(jac.d_mat)})
    torch.set_default_dtype(torch.float32)
    save("pbc_jacobi.npz", **out)


if __name__ == "__main__":
    torch.set_num_threads(8)
    t0 = time.time()
    if len(sys.argv) > 1:  # selected generators only, e.g. `make_golden.py pbc_runs`
        for name in sys.argv[1:]:
            globals()[name]()
        sys.exit(0)
    gen_tables()
    gen_ops()
    mg_test_runs()
    mg_test_synthetic()
    mm_convergence_runs()
    mm_interface_run()
    multigrid_py_runs()
    multigrid_py_training()
    dataset_fixtures()
    recorded_outputs()
    weights()
    pbc_runs()
    print(f"done in {time.time() - t0:.1f}s")
