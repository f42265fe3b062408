"""Lab: per-kernel VGPRs / SGPRs / scratch / occupancy of one source file (hipcc -Rpass-analysis=kernel-resource-usage).
usage: python3 tools/lab/kres.py csrc/FILE.hip [NAME_SUBSTRING ...] [-DDEF ...]"""
import os
import re
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
src = sys.argv[1]
pats = [a for a in sys.argv[2:] if not a.startswith("-D")]
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=on", "-std=c++17", "-Wno-pass-failed",
       f"-I{ROOT}/include", f"-I{ROOT}/multigrid-feanet_amd/csrc", "--cuda-device-only", "-c", src, "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage", *defs]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rec = None, {}
rows = []
for ln in out.splitlines():
    m = re.search(r"remark: +(.*?) \[-Rpass", ln)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        if cur:
            rows.append((cur, rec))
        cur, rec = t.split(":", 1)[1].strip(), {}
    elif ":" in t:
        k, v = t.split(":", 1)
        rec[k.strip()] = v.strip()
if cur:
    rows.append((cur, rec))
for name, r in rows:
    if pats and not any(p in name for p in pats):
        continue
    print(f"{name[:90]:90s} VGPR {r.get('VGPRs', '?'):>4s} AGPR {r.get('AGPRs', '?'):>3s} SGPR {r.get('SGPRs', '?'):>3s} "
          f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4s} occ {r.get('Occupancy [waves/SIMD]', '?')}")
