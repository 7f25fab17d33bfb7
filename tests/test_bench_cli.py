"""bench.py's launcher contract on CPU (no GPU call is made on these paths).

`python bench.py --gpus N` with no WORLD_SIZE in the environment launches N ranks itself
(torch.distributed.run as a child process) — it must refuse loudly, before any GPU call,
when fewer than N devices are visible; a rank whose launcher started a different number of
ranks than --gpus must refuse too.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "SD_BENCH_ONE_DEVICE")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, env=e, timeout=300)


def test_gpus_n_refuses_without_devices():
    r = _run(["--gpus", "2"])
    assert r.returncode == 2, r.stderr
    assert "needs 2 visible GPUs" in r.stderr
    assert r.stdout == ""


def test_rank_refuses_world_mismatch():
    r = _run(["--gpus", "2"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=1" in r.stderr


def test_gpus_zero_is_an_error():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0
