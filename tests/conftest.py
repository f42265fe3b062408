"""Shared pytest setup: registers the `gpu` marker and puts the product package
directory (multigrid-feanet_amd/) and the oracle on sys.path."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "multigrid-feanet_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) and the built libfeanet_hip.so")


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def gold():
    return golden


def pytest_sessionstart(session):
    # keep the in-tree library in sync with csrc/ when a compiler is available (build container);
    # on the GPU box the prebuilt .so from the snapshot is used as is.
    # A failed build ends the session: a green run must never test a stale library.
    if os.path.exists("/opt/rocm/bin/hipcc"):
        from feanet_amd import build
        try:
            build.build(verbose=False)
        except Exception as e:  # pragma: no cover
            pytest.exit(f"feanet_amd build failed: {e}", returncode=1)
