"""bench.py --gpus N on CPU: the launcher starts N ranks itself (no WORLD_SIZE
in the environment, the way the driver calls `python3 bench.py --gpus N`),
the ranks form one process group of exactly N, run the sharded decode loop
(dist_decode.ShardedDecode + timed_run) over a stub host step in place of the
HIP decoder, and rank 0 prints ONE JSON line whose n_gpus, per-rank step
times, scaling mode and gather fields describe those N ranks.  A failing rank
makes the launcher exit non-zero; a rank count that differs from --gpus is
refused."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
LAUNCH_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
              "MASTER_PORT")


def _bench(*args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_ENV}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints, exactly one line
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_starts_n_ranks_strong_headline(n):
    res = _line(_bench("--gpus", str(n), "--stub-step", "--no-cpu-baseline", "--steps", "3",
                       "--warmup", "1"))
    assert res["n_gpus"] == n
    assert res["process_group"] == {"backend": "gloo", "size": n}
    assert len(res["per_rank_ms_per_step"]) == n
    assert max(res["per_rank_ms_per_step"]) == pytest.approx(res["ms_per_step"], rel=1e-3)
    # C3's metric mode: a global batch of 64 split over the ranks
    assert res["scaling"] == "strong"
    assert res["config"]["global_batch"] == 64
    assert res["config"]["batch_per_gpu"] == -(-64 // n)  # rank 0 holds the larger shard
    assert res["value"] == pytest.approx(64 / (res["ms_per_step"] * 1e-3), rel=1e-3)
    g = res["gather"]
    assert g["what"] == "logits" and g["bytes_per_rank"] == res["config"]["batch_per_gpu"] * 50257 * 4
    assert g["alone_ms"] > 0
    # the weak figure rides along: 64 rows on every rank
    w = res["weak_scaling"]
    assert w["global_batch"] == 64 * n and w["batch_per_gpu"] == 64
    assert len(w["per_rank_ms_per_step"]) == n
    assert w["value"] == pytest.approx(64 * n / (w["ms_per_step"] * 1e-3), rel=1e-3)


def test_launcher_weak_config_and_ids_gather():
    res = _line(_bench("--gpus", "2", "--config", "c5", "--gather", "ids", "--stub-step",
                       "--no-cpu-baseline", "--steps", "2", "--warmup", "1"))
    assert res["n_gpus"] == 2 and res["scaling"] == "weak"
    assert res["config"]["global_batch"] == 128 and res["config"]["batch_per_gpu"] == 64
    assert res["gather"]["bytes_per_rank"] == 64 * 4
    assert res["weak_scaling"] is None


def test_launcher_cpu_baseline_on_rank0_at_n2():
    res = _line(_bench("--gpus", "2", "--config", "c1", "--stub-step", "--steps", "2",
                       "--warmup", "1", "--cpu-budget", "2"))
    assert res["n_gpus"] == 2
    cpu = res["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] >= 1


def test_launcher_failing_rank_exits_nonzero():
    r = _bench("--gpus", "3", "--stub-step", "--no-cpu-baseline", "--steps", "2", "--warmup",
               "1", "--stub-fail-rank", "1", timeout=120)
    assert r.returncode != 0
    assert "rank 1 exited" in r.stderr
    assert not r.stdout.strip()


def test_rank_count_must_equal_gpus():
    # an external launcher that started 1 rank while --gpus says 2
    r = _bench("--gpus", "2", "--stub-step", "--no-cpu-baseline",
               env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, timeout=60)
    assert r.returncode != 0
    assert "--gpus 2 but the launcher started 1 rank" in r.stderr


def test_torchrun_launch_and_cpu_baseline_share():
    """The driver's multi-GPU form: torch.distributed.run starts the ranks
    (WORLD_SIZE set, no self-spawn) and sets OMP_NUM_THREADS=1 in each; the
    CPU baseline on rank 0 keeps the 1-GPU job's OpenMP share."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_ENV + ("OMP_NUM_THREADS",)}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), str(ROOT / "bench.py"), "--gpus", "2", "--config", "c1",
                        "--stub-step", "--steps", "2", "--warmup", "1", "--cpu-budget", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    res = _line(r)
    assert res["n_gpus"] == 2 and res["process_group"]["size"] == 2
    cpu = res["cpu_baseline"]
    avail = len(os.sched_getaffinity(0))
    assert cpu["cores"] == min(16, avail), cpu
    assert "torch.distributed.run" in cpu["threads_reason"]


def test_launcher_sigterm_stops_its_ranks():
    """The launcher stopped from outside (the driver's timeout, ^C) takes its
    ranks along instead of leaving them running (a rank blocked in a
    collective would never exit on its own)."""
    import signal
    import time

    import psutil
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_ENV}
    p = subprocess.Popen([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--stub-step",
                          "--no-cpu-baseline", "--steps", "1000000", "--warmup", "1"], cwd=ROOT,
                         env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        kids = []
        for _ in range(100):
            kids = psutil.Process(p.pid).children()
            if len(kids) == 2:
                break
            time.sleep(0.1)
        assert len(kids) == 2, kids
        time.sleep(2)
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) == 128 + signal.SIGTERM
        _, alive = psutil.wait_procs(kids, timeout=15)
        assert not alive, alive
    finally:
        if p.poll() is None:
            p.kill()
