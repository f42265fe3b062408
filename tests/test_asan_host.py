"""AddressSanitizer build of the C ABI's host code (sanitizers): tests/asan/host_checks.cpp
exercises every host-side path that runs without a GPU — layout/workspace queries, LDS sizing and the
argument checks the launchers perform before any device call — with -fsanitize=address on the host
side of every source (hipcc: -Xarch_host; the device code is compiled as for the product).  Skipped
where hipcc is absent."""
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

from conftest import ROOT

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CSRC = os.path.join(ROOT, "multigrid-feanet_amd", "csrc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_host_code_under_asan(tmp_path):
    flags = ["--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-ffp-contract=on", "-Wno-pass-failed",
             "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer",
             f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}"]
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    srcs.append(os.path.join(ROOT, "tests", "asan", "host_checks.cpp"))
    objs = [str(tmp_path / (os.path.basename(s) + ".o")) for s in srcs]

    def cc(pair):
        s, o = pair
        return subprocess.run([HIPCC, *flags, "-c", s, "-o", o], capture_output=True, text=True)

    with ThreadPoolExecutor(min(8, os.cpu_count() or 4)) as ex:
        for r in ex.map(cc, zip(srcs, objs)):
            assert r.returncode == 0, r.stderr[-2000:]
    exe = str(tmp_path / "host_checks")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-fsanitize=address", "-fno-gpu-sanitize", *objs, "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and "asan host checks ok" in r.stdout, (r.stdout + r.stderr)[-3000:]
    assert "AddressSanitizer" not in r.stderr
