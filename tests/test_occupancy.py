"""Register-budget guard for the dominant kernel: the fp64 cycle join must fit 168 VGPRs so three waves
per SIMD stay resident (one round of workgroups at 4097^2: 753 of the 768 slots).  At 175 VGPRs it drops
to two waves per SIMD and the join runs 15 % slower (measured, r02 A/B), with bitwise identical results
— so only this check catches it.  Compiles framed_ops.hip to gfx950 assembly (CPU only)."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_join_fits_three_waves_per_simd(tmp_path):
    csrc = os.path.join(ROOT, "multigrid-feanet_amd", "csrc")
    out = tmp_path / "framed.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-ffp-contract=on", "-std=c++17", "--cuda-device-only",
                    "-S", f"-I{os.path.join(ROOT, 'include')}", f"-I{csrc}", os.path.join(csrc, "framed_ops.hip"),
                    "-o", str(out)], check=True, capture_output=True)
    meta = {}
    name = None
    for line in open(out):
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
        m = re.match(r"\s+\.vgpr_count:\s+(\d+)", line)
        if m and name:
            meta.setdefault(name, {})["vgpr"] = int(m.group(1))
        m = re.match(r"\s+\.vgpr_spill_count:\s+(\d+)", line)
        if m and name:
            meta.setdefault(name, {})["spill"] = int(m.group(1))
    # k_mg_cycle_join<double, MULTI=false, NORM, NT>: the metric configuration's kernels
    joins = {n: v for n, v in meta.items() if n.startswith("_ZN3fea15k_mg_cycle_joinIdLb0E")}
    assert len(joins) == 4, sorted(meta)
    for n, v in joins.items():
        assert v.get("spill", 0) == 0 and v["vgpr"] <= 168, (n, v)
