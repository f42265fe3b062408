"""Register-budget guard for the dominant kernel: the fp64 cycle join must fit 168 VGPRs so three waves
per SIMD stay resident (one round of workgroups at 4097^2: 753 of the 768 slots).  At 175 VGPRs it drops
to two waves per SIMD and the join runs 15 % slower (measured, r02 A/B), with bitwise identical results
— so only this check catches it.  Reads the kernel metadata of the built library's gfx950 code objects
(llvm-objdump --offloading, llvm-readobj --notes; CPU only)."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(ROOT, "multigrid-feanet_amd", "feanet_amd", "libfeanet_hip.so")


def kernel_meta(tmp_path):
    so = tmp_path / "lib.so"
    shutil.copy(LIB, so)
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", str(so)], check=True, capture_output=True, cwd=tmp_path)
    meta, name = {}, None
    for co in sorted(tmp_path.glob("lib.so.*gfx950*")):
        notes = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
        for line in notes.splitlines():
            m = re.match(r"\s+\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
            m = re.match(r"\s+\.(vgpr_count|vgpr_spill_count):\s+(\d+)", line)
            if m and name:
                meta.setdefault(name, {})[m.group(1)] = int(m.group(2))
    return meta


@pytest.mark.skipif(not (os.path.exists(f"{LLVM}/llvm-readobj") and os.path.exists(LIB)),
                    reason="llvm tools or the built library not available")
def test_join_fits_three_waves_per_simd(tmp_path):
    meta = kernel_meta(tmp_path)
    # k_mg_cycle_join<double, MULTI=false, NORM, NT, NTF>: the metric configuration's kernels (NT x NORM,
    # plus the non-temporal right-hand-side loads of the fields beyond the Infinity Cache)
    joins = {n: v for n, v in meta.items() if n.startswith("_ZN3fea15k_mg_cycle_joinIdLb0E")}
    assert len(joins) == 6, sorted(meta)[:20]
    for n, v in joins.items():
        assert v.get("vgpr_spill_count", 0) == 0 and v["vgpr_count"] <= 168, (n, v)
