"""bench.py --gpus N run without a launcher starts N ranks itself (VERDICT 4,
item 1): the driver's `python bench.py --gpus 8` must time 8 GPUs, not one.
CPU only: the ranks join a gloo group and report what they saw
(--spawn-check), and the RCCL default refuses more ranks than GPUs."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "DVO_BENCH_BACKEND")}
    env.update(kw)
    return env


def _run(args, env):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


def test_gpus_2_spawns_two_gloo_ranks():
    p = _run(["--gpus", "2", "--spawn-check"], _env(DVO_BENCH_BACKEND="gloo"))
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    seen = json.loads(lines[0])["spawn_check"]
    assert [s["rank"] for s in seen] == [0, 1]
    assert [s["local_rank"] for s in seen] == [0, 1]
    assert all(s["world"] == 2 for s in seen)
    assert len({s["pid"] for s in seen}) == 2


def test_gpus_beyond_device_count_fails_loudly_with_rccl():
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    p = _run(["--gpus", str(n)], _env())
    assert p.returncode != 0
    assert "needs" in p.stderr and "GPUs" in p.stderr, p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
