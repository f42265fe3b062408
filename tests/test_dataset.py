"""Data.dataset drop-in and the h5py-free HDF5 reader (feanet_amd.h5lite).

Checked against the reference's own data files when /root/reference is present (this container;
skipped elsewhere): every dataset's shape, and the values against raw reads at the offsets SURVEY
§8c lists (the files hold contiguous little-endian float64 blocks), plus the IsoPoisson sample the
golden fixtures were made from.  Nothing here reads the reference at GPU-test time."""
import os

import numpy as np
import pytest
import torch

REF = "/root/reference/Data"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference data files not present")


def raw(path, off, shape):
    return np.fromfile(os.path.join(REF, path), dtype="<f8", count=int(np.prod(shape)), offset=off).reshape(shape)


def test_h5lite_reads_reference_files():
    from feanet_amd.h5lite import File
    with File(os.path.join(REF, "IsoPoisson/poisson2d_33x33.h5")) as h:
        assert sorted(h.keys()) == ["boundary_index", "boundary_value", "rhs", "u"]
        for name, off in (("boundary_index", 2048), ("boundary_value", 873248), ("rhs", 1744448),
                          ("u", 2617696)):
            np.testing.assert_array_equal(np.array(h[name]), raw("IsoPoisson/poisson2d_33x33.h5", off, (100, 33, 33)))
    with File(os.path.join(REF, "TestPoisson/poisson2d_33x33.h5")) as h:
        assert h["material"].shape == (10, 32, 32, 1) and h["solution"].shape == (10, 33, 33)
        np.testing.assert_array_equal(np.array(h["dirich_idx"])[..., 0],
                                      raw("TestPoisson/poisson2d_33x33.h5", 2048, (10, 33, 33)))
        np.testing.assert_array_equal(np.array(h["solution"]), raw("TestPoisson/poisson2d_33x33.h5", 521616, (10, 33, 33)))
    with File(os.path.join(REF, "RHS/poisson2d_rhs_17x17.h5")) as h:
        np.testing.assert_array_equal(np.array(h["train"]), raw("RHS/poisson2d_rhs_17x17.h5", 2048, (1000, 17, 17)))
        np.testing.assert_array_equal(np.array(h["test"]), raw("RHS/poisson2d_rhs_17x17.h5", 2314048, (200, 17, 17)))
        with pytest.raises(KeyError):
            h["nope"]


def test_h5lite_rejects_non_hdf5(tmp_path):
    from feanet_amd.h5lite import File
    p = tmp_path / "x.h5"
    p.write_bytes(b"not hdf5" * 100)
    with pytest.raises(ValueError):
        File(str(p))


def test_datasets_match_reference_semantics(gold):
    from Data.dataset import IsoPoissonDataSet, IsoPoissonPBCDataSet, RHSDataSet, TestPoissonDataSet
    iso = IsoPoissonDataSet(os.path.join(REF, "IsoPoisson/poisson2d_33x33.h5"))
    assert len(iso) == 100
    u, f, bcv, bci = iso[0]
    assert u.shape == (1, 33, 33) and u.dtype == torch.float32
    np.testing.assert_array_equal(f.numpy()[0], raw("IsoPoisson/poisson2d_33x33.h5", 1744448, (100, 33, 33))[0].astype(np.float32))
    g = gold("mg_test_isopoisson33.npz")  # the fixtures the golden runs were made from
    np.testing.assert_array_equal(bcv.numpy()[0], g["boundary_value"][0].astype(np.float32))
    pbc = IsoPoissonPBCDataSet(os.path.join(REF, "IsoPoisson/poisson2d_33x33.h5"))
    assert len(pbc) == 100 and torch.equal(pbc[3], iso[3][1])
    tp = TestPoissonDataSet(os.path.join(REF, "TestPoisson/poisson2d_33x33.h5"))
    items = tp[2]
    assert len(tp) == 10 and len(items) == 7 and all(t.dtype == torch.float64 for t in items)
    assert items[4].shape == (1, 32, 32) and items[0].shape == (1, 33, 33) and items[6].shape == (1, 33, 33)
    rhs = RHSDataSet(os.path.join(REF, "RHS/poisson2d_rhs_17x17.h5"), case="test")
    assert len(rhs) == 200 and rhs[0].shape == (1, 17, 17)
    loader = torch.utils.data.DataLoader(iso, batch_size=8)
    ub, fb, _, _ = next(iter(loader))
    assert ub.shape == (8, 1, 33, 33)
    t2 = IsoPoissonDataSet(os.path.join(REF, "IsoPoisson/poisson2d_33x33.h5"), transform=lambda t: 2 * t)
    assert torch.equal(t2[1][1], 2 * iso[1][1])
