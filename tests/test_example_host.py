"""The C host example (examples/sd_identify.c): the whole identifier hot path driven through
the C ABI from a compiled program with no Python or torch in the process — walk, batched
generate_cas_id from paths, the job's Object decisions with the reference's cursor, and
thumbnail paths.  CPU: it links and loads, and refuses to run without a gfx950 device.
GPU: every row equals the oracle (cas_id, thumbnail path) and the literal job replay
(step, action, owner, per-step counts)."""
import json
import os
import subprocess

import numpy as np
import pytest

from oracle.pyoracle import py_thumbnail_path
from tests.golden.make_golden import replay_identifier_job

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "sd_identify")
LIB = "3f0c6d1e-55aa-4b7c-9e1d-0a1b2c3d4e5f"
ACT = {"created": 0, "linked": 1, "dropped": 2, "not_reached": 3}


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-C", os.path.join(ROOT, "examples"), "-s"], check=True)
    return EXE


def test_example_links_and_refuses_without_gpu(exe, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the GPU test covers the example")
    (tmp_path / "a").write_bytes(b"x")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1
    assert "sd_cas_ctx_create: -5" in r.stderr and "no HIP device" in r.stderr


@pytest.mark.gpu
def test_example_job_vs_oracle_and_replay(exe, oracle, tmp_path):
    rng = np.random.default_rng(21)
    d = tmp_path / "lib"
    (d / "sub").mkdir(parents=True)
    blobs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in [3, 4096, 102400, 250_000, 3_000_000]]
    for i in range(230):
        p = d / ("sub" if i % 3 == 0 else ".") / f"f{i:04d}"
        if i % 29 == 3:
            p.write_bytes(b"")  # indexed with size 0: not an orphan row of the job
        elif rng.random() < 0.4:
            p.write_bytes(blobs[int(rng.integers(0, len(blobs)))])
        else:
            p.write_bytes(rng.integers(0, 256, int(rng.integers(1, 400_000)), dtype=np.uint8).tobytes())
    bad = d / "f0100"  # unreadable for a non-root user: an ERROR row, dropped from its step
    os.chmod(bad, 0)
    data_dir = str(tmp_path / "node")
    r = subprocess.run([exe, str(d), "7", data_dir, LIB], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines()]
    files = [x for x in lines if "path" in x]
    steps = [x for x in lines if "path" not in x]
    paths = sorted(str(p) for p in d.rglob("*") if p.is_file())
    assert [x["path"] for x in files] == paths
    # the job's rows: file_paths indexed with size 0 are not orphans of the job
    # (orphan_path_filters, file_identifier_job.rs:264)
    rows = []
    for x in files:
        if os.path.getsize(x["path"]) == 0:
            assert x["row"] is None and x["action"] == "not_queried"
        else:
            assert x["row"] == len(rows)
            rows.append(x)
    keys, states = [], []
    for x in rows:
        size = os.path.getsize(x["path"])
        assert x["size"] == size
        if not os.access(x["path"], os.R_OK):
            keys.append(0); states.append(2)
            assert x["cas_id"] is None and x["errno"] == 13
        else:
            want = oracle.generate_cas_id(x["path"], size)
            assert x["cas_id"] == want, x["path"]
            assert x["thumbnail"] == py_thumbnail_path(data_dir, want, LIB)
            keys.append(int(want, 16)); states.append(0)
    step, obj, act, counts = replay_identifier_job(keys, states, 7)
    for i, x in enumerate(rows):
        assert ACT[x["action"]] == act[i], i
        assert (x["step"] if x["step"] is not None else 0xFFFFFFFF) == step[i], i
        assert (x["object"] if x["object"] is not None else 0xFFFFFFFF) == obj[i], i
    assert [(s["total_created"], s["total_linked"]) for s in steps] == [tuple(c) for c in counts]


VEXE = os.path.join(ROOT, "examples", "sd_validate")


def test_validate_example_refuses_without_gpu(exe, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the GPU test covers the example")
    (tmp_path / "a").write_bytes(b"x")
    r = subprocess.run([VEXE, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "sd_cas_ctx_create: -5" in r.stderr


@pytest.mark.gpu
def test_validate_example_vs_oracle(exe, oracle, tmp_path):
    """examples/sd_validate.c: the validator job over a directory from a compiled host —
    one sd_cas_file_checksums call; every integrity_checksum equals the oracle's
    file_checksum (hash.rs:11-25), an unreadable file reports errno 13."""
    rng = np.random.default_rng(22)
    d = tmp_path / "lib"
    (d / "sub").mkdir(parents=True)
    for i in range(120):
        p = d / ("sub" if i % 4 == 0 else ".") / f"v{i:03d}"
        L = 0 if i % 37 == 5 else int(rng.integers(1, 3_000_000 if i % 10 else 70_000_000))
        p.write_bytes(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
    bad = d / "v050"
    os.chmod(bad, 0)
    r = subprocess.run([VEXE, str(d)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rows = [json.loads(x) for x in r.stdout.splitlines()]
    assert [x["path"] for x in rows] == sorted(str(p) for p in d.rglob("*") if p.is_file())
    for x in rows:
        assert x["size"] == os.path.getsize(x["path"])
        if not os.access(x["path"], os.R_OK):
            assert x["integrity_checksum"] is None and x["errno"] == 13
        else:
            assert x["errno"] == 0 and x["integrity_checksum"] == oracle.file_checksum(x["path"]), x["path"]
