"""Product setup code (feanet_amd.mesh_setup: vectorised pattern maps, stencil/mass tables)
against golden tables generated from the reference.  CPU only, bit-exact."""
import pytest
import numpy as np

from feanet_amd import mesh_setup as ms
from oracle import feanet_oracle as orc


def test_stencils_bit_exact(gold):
    t = gold("tables.npz")
    np.testing.assert_array_equal(ms.stencil_table(None), t["square_kernel"])
    np.testing.assert_array_equal(ms.stencil_table((1, 20)), t["iface0_kernel_65"])
    np.testing.assert_array_equal(ms.stencil_table((3, 7)), t["iface0_prop3_7_kernel"])


def test_pattern_maps_bit_exact(gold):
    t = gold("tables.npz")
    for shape in (0, 1):
        for n in (5, 9, 17, 33, 65, 129):
            np.testing.assert_array_equal(ms.interface_pattern_map(n, shape), t[f"iface{shape}_pid_{n}"],
                                          err_msg=f"shape={shape} N={n}")


def test_pattern_maps_match_oracle_large():
    # beyond the reference-generated sizes: the loop oracle and the vectorised product agree
    for shape in (0, 1):
        _, pid = orc.interface_mesh(257, (1, 20), shape)
        np.testing.assert_array_equal(ms.interface_pattern_map(257, shape), pid)


def test_c3_maps_fixture_is_oracle(gold):
    """Config C3 (2049^2 two-material): the oracle's element/node loop at the full size equals the
    fixture the C3 GPU test builds its oracle hierarchy from, and the product's vectorised builder
    equals the fixture on every level of the hierarchy (2049^2 .. 3^2).  ~70 s (the loop)."""
    maps = gold("c3_pattern_maps.npz")
    ktab, pid = orc.interface_mesh(2049, (1, 20), 0)
    np.testing.assert_array_equal(pid, maps["pid_2049"])
    np.testing.assert_array_equal(ktab, maps["ktab"])
    np.testing.assert_array_equal(ms.stencil_table((1, 20)), maps["ktab"])
    N = 2049
    while N >= 3:
        np.testing.assert_array_equal(ms.interface_pattern_map(N, 0), maps[f"pid_{N}"], err_msg=f"N={N}")
        N = (N + 1) // 2


def test_mass_stencil(gold):
    t = gold("tables.npz")
    for n in (2, 4, 16, 32, 64, 128, 4096):
        np.testing.assert_array_equal(ms.mass_stencil(2 / n), t[f"fnet_{n}"])


def test_omega_over_d(gold):
    for case in ("poisson", "iface0"):
        for dt, npdt in (("f32", np.float32), ("f64", np.float64)):
            g = gold(f"ops_{case}_{dt}_n16.npz")
            omd = ms.omega_over_d(g["ktab"], 2 / 3., npdt)
            # reference d_mat per node, and omega/d_mat the way torch evaluates it
            d = g["d_mat"][0, 0]
            ref = (np.reciprocal(d.astype(npdt)) * npdt(2 / 3.)).astype(npdt)
            np.testing.assert_array_equal(omd[g["pid"].astype(np.int64)], ref)


def test_large_pattern_map_fast():
    import time
    t0 = time.time()
    pid = ms.interface_pattern_map(2049, 0)
    assert time.time() - t0 < 5.0
    assert pid.shape == (2049, 2049) and pid.max() < 16


def test_vtk_export_roundtrip(tmp_path):
    """MeshCenterInterface(outfile=...) / save_mesh without meshio: legacy binary VTK with the
    reference's points, quad cells and element phases (FEANet/mesh.py:44-60, 62-68, 119-120)."""
    from FEANet.mesh import MeshCenterInterface, MeshSquare, read_vtk_legacy
    from feanet_amd import mesh_setup as ms
    N = 17
    p = tmp_path / "plate.vtk"
    m = MeshCenterInterface(nnode_edge=N, shape=1, outfile=str(p))
    d = read_vtk_legacy(str(p))
    np.testing.assert_array_equal(d["points"], m.points)
    np.testing.assert_array_equal(d["cells"], m.cells)
    assert (d["types"] == 9).all()
    np.testing.assert_array_equal(d["CELL_DATA"]["Phase"], ms.element_phase(N, 1).reshape(-1))
    q = tmp_path / "sq.vtk"
    sq = MeshSquare(nnode_edge=N)
    u = np.linspace(0, 1, N * N)
    sq.save_mesh(str(q), point_data={"u": u})
    d = read_vtk_legacy(str(q))
    assert (d["CELL_DATA"]["Phase"] == 0).all()
    np.testing.assert_array_equal(d["POINT_DATA"]["u"], u)


@pytest.mark.parametrize("prop", [(1, 20), (1, 5), (3, 7)])
@pytest.mark.parametrize("shape", [0, 1])
def test_stiffness_mirror_symmetry(prop, shape):
    """The framed two-material kernels take every node's nine stiffness weights from its own pattern's table row,
    mirrored (tap 8 - t), where KNet weighs tap t by the neighbour's pattern (FEANet/model.py:22-30): equal bit for bit
    because K is a symmetric FE stiffness — on every level map of both inclusion shapes; a random table is not."""
    from feanet_amd import mesh_setup as ms
    kt = ms.stencil_table(prop)
    for N in (5, 9, 33, 65, 129, 257):
        assert ms.stencil_mirror_mismatches(kt, ms.interface_pattern_map(N, shape, 2.0)) == 0, N
    rng = np.random.default_rng(1)
    assert ms.stencil_mirror_mismatches(rng.standard_normal((16, 9)), ms.interface_pattern_map(65, shape, 2.0)) > 0
