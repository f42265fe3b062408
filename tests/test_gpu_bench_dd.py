"""The multi-GPU bench line end to end: bench.py under torch.distributed.run with two ranks on the one GPU
(gloo, device halos staged through the host), as the driver's N > 1 runs launch it (they use RCCL, one GPU
per rank).  The line must carry its strong-scaling base point and a dd_parity record in which every rank's
owned block equals the single-GPU solver's bitwise."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    p = sk.getsockname()[1]
    sk.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("ranks,grid,extra", [(2, None, []), (4, "2x2", []),
                                              (4, "2x2", ["--problem", "interface", "--smoother", "hjac"])])
def test_bench_dd_line_parity(ranks, grid, extra):
    """The N > 1 line over gloo: every mode bitwise; also the decomposed two-material problem with the learned
    smoother (--problem interface --smoother hjac)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(ranks), "--steps", "3", "--warmup", "1", "--backend", "gloo", "--global-n", "1024",
           "--kernel-reps", "2"] + (["--grid", grid] if grid else []) + extra
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == ranks and rec["scaling"] == "strong" and rec["config"]["mode"] == "dd"
    par = rec["dd_parity"]
    assert par["bitwise_equal"] and par["max_abs_diff"] == 0.0, par
    base = rec["single_gpu_same_grid"]
    assert base["ms_per_step"] > 0 and base["workload"].startswith("1025x1025")
    # every DD mode gloo can run (segment graphs, level-0 halo overlapped, split join) timed on the live
    # communicator, each bitwise the single-GPU solver over its eager / captured / replayed runs; the headline is
    # the fastest of them
    modes = rec["dd_modes"]
    timed = [m for m in modes if m["status"] == "ok"]
    assert len(timed) >= 3, modes
    assert {m["mode"] for m in timed} >= {"segments", "segments+overlap_l0", "segments+split_join"}
    for m in timed:
        assert m["ms_per_step"] > 0 and m["dd_parity"]["bitwise_equal"], m
        assert m["dd_parity"]["repeats"] == 3 and m["dd_parity"]["max_abs_diff"] == 0.0, m
    best = min(timed, key=lambda m: m["ms_per_step"])
    assert rec["headline_mode"] == best["mode"] and rec["ms_per_step"] == best["ms_per_step"]
    assert rec["config"]["dd_mode"]["mode"] == best["mode"]
    if extra:
        assert "interface" in rec["config"]["workload"] and "HRelax" in rec["config"]["workload"]
        assert base["workload"].startswith("1025x1025 interface")


@pytest.mark.timeout(300)
def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` with no launcher starts the two ranks itself (torch.distributed.run as a child
    process), forwards rank 0's one JSON line and records the decomposition mode it ran."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--backend", "gloo", "--global-n", "1024", "--kernel-reps", "2"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["mode"] == "dd"
    assert rec["dd_parity"]["bitwise_equal"], rec["dd_parity"]
    dm = rec["config"]["dd_mode"]
    assert dm["backend"] == "gloo" and dm["cycle_graphs"].startswith("segments")  # gloo is never captured
    assert not any(m["capture_requested"] for m in rec["dd_modes"])
    timed = [m for m in rec["dd_modes"] if m["status"] == "ok"]
    assert len(timed) >= 3 and all(m["dd_parity"]["bitwise_equal"] for m in timed), rec["dd_modes"]
