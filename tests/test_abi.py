"""The C-ABI library builds, loads on a CPU-only host and exports every entry point declared in
include/feanet_hip.h (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def header_functions():
    src = open(os.path.join(ROOT, "include", "feanet_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fea_[a-z0-9_]+)\s*\(", src)))


def test_header_lists_both_families():
    names = header_functions()
    assert "fea_knet_apply_f64" in names and "fea_mg_prolong_sweep_f32" in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol():
    from feanet_amd import _lib
    lib = _lib.lib()
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, f"not exported: {missing}"
    assert sorted(_lib.exported_symbols()) == header_functions()


def test_host_only_queries():
    from feanet_amd import _lib
    assert _lib.lib().fea_abi_version() == _lib.ABI_VERSION
    for H, W, esz in [(3, 3, 8), (5, 5, 8), (4097, 4097, 8), (1025, 1025, 4), (8193, 8193, 8), (517, 4097, 8),
                      (9, 100, 4)]:
        ld, bs = _lib.mg_layout(H, W, esz)
        A = 128 // esz
        assert ld % A == 0 and ld >= W + A and bs == (H + 2) * ld
    with pytest.raises(ValueError):
        _lib.mg_layout(2, 100, 8)       # fewer than 3 rows
    assert _lib.norm_workspace_bytes(2, 4097, 4097) >= 2 * 65 * 129 * 8


def test_ops_refuse_cpu_tensors():
    import torch
    from feanet_amd import ops
    with pytest.raises(RuntimeError, match="MI355X"):
        ops.knet_apply(torch.zeros(1, 1, 5, 5), torch.zeros(1, 9))


def test_no_oracle_in_product():
    """Nothing under multigrid-feanet_amd/ may import the oracle (test infrastructure only)."""
    pkg = os.path.join(ROOT, "multigrid-feanet_amd")
    for dp, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dp, fn)).read()
                assert "feanet_oracle" not in txt and "from oracle" not in txt, fn
