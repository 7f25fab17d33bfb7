"""Host-side checks of the round-6 measurement tools (no GPU): the rehearsal checker pulls the
bench line out of a committed one-GPU N-rank rehearsal log (gloo chatter around it) and
passes it, and fails a line whose exchange overflowed."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "rehearsal_check.py")


def run(log, n):
    return subprocess.run([sys.executable, TOOL, log, str(n)], capture_output=True, text=True)


def test_rehearsal_check_on_committed_logs(tmp_path):
    for n in (2, 4, 8):
        src = os.path.join(ROOT, "profiles", "r06", "final", f"bench_n{n}_rehearsal.log")
        log = tmp_path / f"n{n}.log"
        log.write_text(open(src, errors="replace").read())
        r = run(str(log), n)
        assert r.returncode == 0, r.stdout + r.stderr
        d = json.loads(r.stdout)
        assert d["ok"] and d["n_gpus"] == n and d["capacity_per_peer"] > 0
        assert json.load(open(tmp_path / f"n{n}.json"))["n_gpus"] == n


def test_rehearsal_check_rejects_overflow_and_wrong_n(tmp_path):
    src = os.path.join(ROOT, "profiles", "r06", "final", "bench_n2_rehearsal.json")
    line = json.load(open(src))
    assert run_line(tmp_path, line, 4).returncode == 1  # n_gpus mismatch
    bad = json.loads(json.dumps(line).replace('"timed_steps_overflowed": 0', '"timed_steps_overflowed": 3'))
    r = run_line(tmp_path, bad, 2)
    assert r.returncode == 1 and not json.loads(r.stdout)["checks"]["timed_steps_overflowed_0"]


def run_line(tmp_path, line, n):
    log = tmp_path / "x.log"
    log.write_text("[Gloo] Rank 0 is connected to 1 peer ranks.\n" + json.dumps(line) + "\n")
    return run(str(log), n)
