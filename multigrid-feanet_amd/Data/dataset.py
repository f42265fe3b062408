"""Dataset readers of the reference (Data/dataset.py:6-104), same class names, constructor arguments,
__len__/__getitem__ results and dtypes, so the notebooks' `from Data.dataset import ...` lines run
unchanged with this package first on sys.path.

Differences from the reference, none visible to its callers:
  * HDF5 is read with h5py when it is installed, otherwise with feanet_amd.h5lite (h5py is absent in
    this image; the reference's files are plain contiguous datasets);
  * torchvision's ToTensor is restated (`to_tensor`): an H x W array becomes [1, H, W], an H x W x C
    array [C, H, W], dtype kept (the reference's arrays are float, which ToTensor does not rescale).
Samples are CPU tensors, as in the reference; move them to the GPU (or set the default device) before
handing them to the FEANet operators.
"""
import numpy as np
import torch
from torch.utils.data import Dataset

try:  # the reference's reader when present
    import h5py

    def _open(path):
        return h5py.File(path, "r")
except ImportError:  # pragma: no cover - h5py is not installed in this image
    from feanet_amd.h5lite import File as _open


def to_tensor(a):
    """torchvision.transforms.ToTensor on a float ndarray: HxW -> 1xHxW, HxWxC -> CxHxW."""
    a = np.asarray(a)
    if a.ndim == 2:
        a = a[:, :, None]
    return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))


def _read(path, names, dtype):
    h5 = _open(path)
    try:
        return [np.array(h5[n], dtype=dtype) for n in names]
    finally:
        h5.close()


class _Base(Dataset):
    def __init__(self, transform=None, target_transform=None):
        self.totensor = to_tensor
        self.transform = transform
        self.target_transform = target_transform

    def _t(self, a):
        t = self.totensor(a)
        return self.transform(t) if self.transform else t


class RHSDataSet(_Base):
    """Right-hand sides, `case` = 'train' or 'test' (Data/dataset.py:6-24)."""

    def __init__(self, h5file, case='train', transform=None, target_transform=None):
        super().__init__(transform, target_transform)
        (self.data,) = _read(h5file, [case], np.float32)

    def __len__(self):
        return self.data.shape[0]

    def __getitem__(self, idx):
        return self._t(self.data[idx])


class IsoPoissonDataSet(_Base):
    """u, f, bc_value, bc_index (Data/dataset.py:26-51); returns (u, f, bc_value, bc_index)."""

    def __init__(self, h5file, transform=None, target_transform=None):
        super().__init__(transform, target_transform)
        self.bc_index, self.bc_value, self.f, self.u = _read(
            h5file, ["boundary_index", "boundary_value", "rhs", "u"], np.float32)

    def __len__(self):
        return self.f.shape[0]

    def __getitem__(self, idx):
        return (self._t(self.u[idx]), self._t(self.f[idx]), self._t(self.bc_value[idx]),
                self._t(self.bc_index[idx]))


class IsoPoissonPBCDataSet(_Base):
    """Right-hand sides of the periodic problem (Data/dataset.py:53-69)."""

    def __init__(self, h5file, transform=None, target_transform=None):
        super().__init__(transform, target_transform)
        (self.f,) = _read(h5file, ["rhs"], np.float32)

    def __len__(self):
        return self.f.shape[0]

    def __getitem__(self, idx):
        return self._t(self.f[idx])


class TestPoissonDataSet(_Base):
    """Dirichlet/Neumann data, material, source, solution in float64 (Data/dataset.py:71-104)."""

    def __init__(self, h5file, transform=None, target_transform=None):
        super().__init__(transform, target_transform)
        (self.dirich_idx, self.dirich_value, self.traction_idx, self.traction_value, self.material, self.source,
         self.solution) = _read(h5file, ["dirich_idx", "dirich_value", "neumann_idx", "neumann_value", "material",
                                         "source", "solution"], np.double)

    def __len__(self):
        return self.source.shape[0]

    def __getitem__(self, idx):
        return (self._t(self.dirich_idx[idx]), self._t(self.dirich_value[idx]), self._t(self.traction_idx[idx]),
                self._t(self.traction_value[idx]), self._t(self.material[idx]), self._t(self.source[idx]),
                self._t(self.solution[idx]))
