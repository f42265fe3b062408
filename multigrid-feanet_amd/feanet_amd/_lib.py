"""ctypes binding of libfeanet_hip.so (C ABI: include/feanet_hip.h).

The product path has no CPU fallback: if the library is missing or no HIP device is present,
every op raises.  `torch` is imported first so the library binds to the HIP runtime torch
loaded (libamdhip64.so.7), not a second copy.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load)

from .build import LIB

_IN_TREE = LIB

ABI_VERSION = 3

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
F32 = ctypes.c_float
F64 = ctypes.c_double

# name -> argtypes (the _f32/_f64 pairs share a signature up to the scalar type S)
_SIGS = {
    "knet_apply": [P, P, P, P, I, I, I, I, P],
    "split_x": [P, P, P, I, I, I, I, P],
    "jacobi_sweep": [P, P, P, P, P, P, I, P, LL, P, LL, I, I, I, P],
    "residual": [P, P, P, P, P, I, I, I, I, P],
    "jacobi_sweep_pbc": [P, P, P, P, P, I, I, P],
    "pbc_pad": [P, P, I, I, I, I, P],
    "restrict": [P, I, P, P, P, I, "S", I, I, I, P],
    "prolong": [P, I, P, P, P, P, I, "S", I, I, I, P],
    "residual_norm": [P, P, P, P, I, P, P, I, I, I, P],
    # adjoints (autograd)
    "knet_apply_adj": [P, P, P, P, I, I, I, I, P],
    "jacobi_sweep_adj": [P, P, P, P, P, P, I, P, LL, I, I, I, P],
    "restrict_adj": [P, I, P, P, P, I, "S", I, I, I, P],
    "prolong_adj": [P, I, P, P, P, I, "S", I, I, I, P],
    "transfer_weight_grad": [P, I, P, I, I, I, "S", P, P, I, I, I, P],
    "stencil_weight_grad": [P, P, P, I, "S", P, P, I, I, I, P],
    # framed level ops: (..., B, H, W, ld, bstride[, ldc, bstridec], stream)
    "mg_pack": [P, P, P, LL, P, LL, I, I, I, I, LL, P],
    "mg_unpack": [P, P, I, I, I, I, LL, P],
    "mg_sweep": [P, P, P, P, P, P, I, I, I, I, I, LL, P],
    "mg_residual_restrict": [P, P, P, P, P, P, P, I, P, I, "S", I, I, I, I, LL, I, LL, P],
    "mg_zero_restrict2": [P, P, P, P, P, P, P, I, P, I, "S", I, I, I, I, LL, I, LL, I, LL, P],
    "mg_zero_restrict2_send": [P, P, P, P, P, P, P, I, P, I, "S", I, I, I, I, LL, I, LL, I, LL, P, I, I, I, I, P],
    "mg_zero_restrict_send": [P, P, P, P, P, I, P, I, "S", I, I, I, I, LL, I, LL, P, I, I, I, I, P],
    "mg_sweep_restrict": [P, P, P, P, P, P, P, I, P, I, "S", I, I, I, I, LL, I, LL, P, P, P, P],
    "mg_prolong_sweep": [P, P, P, P, P, P, P, P, I, P, I, "S", I, I, I, I, LL, I, LL, P],
    "mg_prolong2": [P, P, P, P, P, P, P, P, P, I, P, I, "S", I, I, I, I, LL, I, LL, I, LL, P],
    "mg_prolong_add": [P, P, P, P, P, I, "S", I, I, I, I, LL, I, LL, P],
    "mg_residual_norm": [P, P, P, P, I, P, P, I, I, I, I, LL, I, I, I, I, P],
    "mg_cycle_join": [P, P, P, P, P, P, P, P, P, I, P, I, P, I, "S", "S", I, I, I, I, LL, I, LL, P, P, P, P],
    "mg_cycle_join_rects": [P, P, P, P, P, P, P, P, P, I, P, I, P, I, "S", "S", I, I, I, I, LL, I, LL, I, P, P],
    "mg_hsweep": [P, P, P, P, P, P, P, I, P, I, I, I, I, I, LL, P],
    "mg_hsweep_restrict": [P, P, P, P, P, P, P, P, I, P, I, P, I, "S", I, I, I, I, LL, I, LL, P],
    "mg_prolong_hsweep": [P, P, P, P, P, P, P, P, P, I, P, I, P, I, "S", I, I, I, I, LL, I, LL, P],
    "mg_coarse_tail": [P, P, I, I, I, I, LL, P, P, P, I, P, P, "S", "S", I, I, I, I, P],
    "mg_coarse_tail_ext": [P, P, I, I, I, LL, I, P, P, I, P, P, "S", "S", I, P],
    "mg_hjac_tail": [P, P, I, I, I, I, LL, P, P, P, I, P, P, P, I, "S", "S", I, I, I, P],
    # several coarse levels per launch (pointer arrays: ptr_array())
    "mg_mid_down": [P, P, I, I, I, I, P, P, I, P, I, "S", I, I, P],
    "mg_mid_down_gathered": [P, P, I, I, I, I, P, P, I, P, I, "S", I, I, P, I, I, I, I, P],
    "mg_mid_up": [P, P, P, P, I, I, I, I, P, P, I, P, I, "S", I, I, P],
    "mg_hmid_down": [P, P, P, I, I, I, P, P, I, P, I, P, I, "S", I, P],
    "mg_hmid_up": [P, P, P, P, P, I, I, I, P, P, I, P, I, P, I, "S", I, P],
}
_EXTRA = {
    "fea_abi_version": ([], I),
    "fea_mg_layout": ([I, I, I, ctypes.POINTER(I), ctypes.POINTER(LL)], I),
    "fea_norm_workspace_bytes": ([I, I, I], ctypes.c_size_t),
    "fea_mg_join_norm_parts": ([I, I, I, I], LL),
    "fea_norm_append": ([P, LL, LL, I, I, P, P, P], I),
    "fea_mg_coarse_tail_lds_bytes": ([I, I, I, I, I], ctypes.c_size_t),
    "fea_mg_hjac_tail_lds_bytes": ([I, I, I, I, I], ctypes.c_size_t),
    "fea_mg_mid_lds_bytes": ([I, I, I, I, I, I], LL),
    "fea_mg_hmid_lds_bytes": ([I, I, I, I, I], LL),
    "fea_interface_pattern_map": ([P, LL, I, I, F64, P], I),
    "fea_dd_copy_blocks": ([P, I, I, I, P], I),
    "fea_dd_copy_rects": ([P, I, I, P], I),
    "fea_stencil_weight_grad_ws_bytes_f32": ([I, I, I, I], ctypes.c_size_t),
    "fea_stencil_weight_grad_ws_bytes_f64": ([I, I, I, I], ctypes.c_size_t),
    "fea_transfer_weight_grad_ws_bytes_f32": ([I, I, I, I], ctypes.c_size_t),
    "fea_transfer_weight_grad_ws_bytes_f64": ([I, I, I, I], ctypes.c_size_t),
}

_lib = None


def exported_symbols():
    """Every symbol the library must export (== every function declared in feanet_hip.h)."""
    names = list(_EXTRA)
    for base in _SIGS:
        names += [f"fea_{base}_f32", f"fea_{base}_f64"]
    return names


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        raise RuntimeError(f"feanet_amd: {LIB} is missing; run `python -m feanet_amd.build` "
                           "(there is no CPU fallback for the HIP path)")
    L = ctypes.CDLL(LIB)  # (A/B builds of tools/lab replace the module attribute LIB: tools/lab/with_lib.py)
    lab = os.path.abspath(LIB) != os.path.abspath(_IN_TREE)  # an older lab build may lack newer entry points

    def sym(name):
        if lab and not hasattr(L, name):
            return None
        return getattr(L, name)
    for name, (args, res) in _EXTRA.items():
        fn = sym(name)
        if fn is not None:
            fn.argtypes = args
            fn.restype = res
    for base, args in _SIGS.items():
        for suf, S in (("f32", F32), ("f64", F64)):
            fn = sym(f"fea_{base}_{suf}")
            if fn is not None:
                fn.argtypes = [S if a == "S" else a for a in args]
                fn.restype = I
    if L.fea_abi_version() != ABI_VERSION:
        raise RuntimeError("feanet_amd: libfeanet_hip.so ABI version mismatch; rebuild it")
    _lib = L
    return L


def call(name, dtype, *args):
    """Invoke fea_<name>_{f32,f64}; raise RuntimeError on a nonzero return (FEA_EINVAL or hipError_t)."""
    suf = {torch.float32: "f32", torch.float64: "f64"}.get(dtype)
    if suf is None:
        raise TypeError(f"feanet_amd: unsupported dtype {dtype} (float32/float64 only)")
    fn = getattr(lib(), f"fea_{name}_{suf}")
    rc = fn(*[a.ptr if isinstance(a, PtrArray) else a for a in args])
    if rc != 0:
        what = "invalid arguments" if rc == -1 else f"hipError_t {rc}"
        raise RuntimeError(f"feanet_amd: fea_{name}_{suf} failed ({what})")


def call_raw(name, *args):
    """Invoke a dtype-free entry point fea_<name> (e.g. norm_append); RuntimeError on a nonzero return."""
    rc = getattr(lib(), f"fea_{name}")(*args)
    if rc != 0:
        raise RuntimeError(f"feanet_amd: fea_{name} failed ({'invalid arguments' if rc == -1 else f'hipError_t {rc}'})")


def join_norm_parts(B, H, W, elem_size):
    """Per-sample partial sums the cycle join writes in its deferred-norm mode."""
    return int(lib().fea_mg_join_norm_parts(B, H, W, elem_size))


def mg_layout(H, W, elem_size):
    """(ld, bstride) of the framed layout of an H x W grid."""
    ld = I()
    bs = LL()
    if lib().fea_mg_layout(H, W, elem_size, ctypes.byref(ld), ctypes.byref(bs)) != 0:
        raise ValueError(f"feanet_amd: unsupported level size {H} x {W} (need H, W >= 3)")
    return ld.value, bs.value


TAIL_LDS_LIMIT = 160 * 1024 - 1024


def coarse_tail_lds_bytes(Ht, Wt, nlev, elem_size, multi):
    return int(lib().fea_mg_coarse_tail_lds_bytes(Ht, Wt, nlev, elem_size, int(bool(multi))))


def hjac_tail_lds_bytes(Ht, Wt, nlev, elem_size, multi):
    return int(lib().fea_mg_hjac_tail_lds_bytes(Ht, Wt, nlev, elem_size, int(bool(multi))))


def weight_grad_ws_bytes(C, B, Hc, Wc):
    return int(lib().fea_transfer_weight_grad_ws_bytes_f64(C, B, Hc, Wc))


def stencil_grad_ws_bytes(ntab, B, H, W):
    return int(lib().fea_stencil_weight_grad_ws_bytes_f64(ntab, B, H, W))


def mid_lds_bytes(up, k, TR, TC, elem_size, multi):
    return int(lib().fea_mg_mid_lds_bytes(int(bool(up)), k, TR, TC, elem_size, int(bool(multi))))


def hmid_lds_bytes(up, T, nlayers, elem_size, multi):
    return int(lib().fea_mg_hmid_lds_bytes(int(bool(up)), T, nlayers, elem_size, int(bool(multi))))


class PtrArray:
    """A C array of device pointers (const T* const*) for the mid-level entry points; keeps the
    ctypes array alive as long as the launch plan that holds it."""

    def __init__(self, ptrs):
        self.arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
        self.ptr = ctypes.cast(self.arr, ctypes.c_void_p).value

    def __repr__(self):
        return f"PtrArray({list(self.arr)})"


def norm_workspace_bytes(B, H, W):
    return int(lib().fea_norm_workspace_bytes(B, H, W))
