"""The host gather pool (spacedrive_amd/csrc/ctx_internal.h HostPool: the persistent workers
behind every path gather) exercised on the CPU: 4,000 calls with random worker counts, back to
back and across pauses that park the workers; every item processed exactly once, the caller's
share run once, no deadlock (the run is under a time limit); the threads' private descriptor
tables (round 6): no copy of the caller's pipe, own files readable, the pipe's EOF intact."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "spacedrive_amd", "csrc")


def test_host_pool(tmp_path):
    exe = str(tmp_path / "pool_test")
    cc = ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-pthread", "-I", CSRC,
          os.path.join(ROOT, "tests", "native", "pool_test.cpp"), "-o", exe]
    if not os.path.exists(cc[0]):
        pytest.skip("hipcc not found")
    subprocess.run(cc, check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "pool ok" in r.stdout, r.stdout + r.stderr
