"""bench.py's command line before any GPU work (CPU suite): a launcher whose WORLD_SIZE disagrees with --gpus is
refused with a non-zero exit, so a driver line can never silently report a different rank count."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and r.stdout.strip() == ""


def test_rank_blocked_in_a_collective_exits_nonzero():
    """A rank blocked in a collective (here: rank 1 never enters the barrier rank 0 waits in, gloo, CPU) ends
    `bench.py --gpus 2` non-zero within the phase limit, naming the rank and the phase — the same process-group
    timeout and PhaseGuard every multi-rank GPU run uses, so a stuck RCCL step cannot outlive the driver's window."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--selftest-hang", "6", "--launch-timeout", "200"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=280)
    took = time.monotonic() - t0
    assert r.returncode != 0, r.stderr[-2000:]
    assert took < 150, took  # the 6 s phase limit, plus interpreter / torch start-up of three processes
    assert "phase 'selftest: barrier that rank 1 skips'" in r.stderr and "rank " in r.stderr, r.stderr[-2000:]
    assert r.stdout.strip() == ""
