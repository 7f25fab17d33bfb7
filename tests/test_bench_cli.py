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


def test_visible_gpus_from_kfd_topology(tmp_path, monkeypatch):
    """spawn_ranks counts GPUs from the KFD topology (no HIP call in the parent): GPU nodes
    have a non-zero gfx_target_version, the CPU node 0; the *_VISIBLE_DEVICES lists narrow it."""
    sys.path.insert(0, ROOT)
    import bench
    for i, ver in enumerate([0, 90500, 90500, 90500]):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 0\ngfx_target_version {ver}\nsimd_count 1024\n")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert bench.visible_gpus(str(tmp_path)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert bench.visible_gpus(str(tmp_path)) == 1
    assert bench.visible_gpus(str(tmp_path / "none")) == 0


def test_cpu_baseline_threads(monkeypatch):
    """The CPU baseline's thread count is the whole node's share: an explicit
    override, else OMP_NUM_THREADS (the box's per-GPU share) x n_gpus — or 16 x n_gpus when
    OMP_NUM_THREADS is 1 or unset (torchrun's default for its workers must not shrink the
    baseline to one core) — capped by the process's affinity mask."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv("SD_CPU_BASELINE_THREADS", raising=False)
    for cores in (200, 96, 8):
        monkeypatch.setattr(os, "sched_getaffinity", lambda pid, c=cores: set(range(c)))
        monkeypatch.setenv("OMP_NUM_THREADS", "16")
        assert bench.cpu_threads(1) == min(cores, 16)
        assert bench.cpu_threads(8) == min(cores, 128)   # never one GPU's 16-core share
        monkeypatch.setenv("OMP_NUM_THREADS", "1")
        assert bench.cpu_threads(1) == min(cores, 16)
        assert bench.cpu_threads(8) == min(cores, 128)
        monkeypatch.delenv("OMP_NUM_THREADS")
        assert bench.cpu_threads(4) == min(cores, 64)
    monkeypatch.setenv("SD_CPU_BASELINE_THREADS", "3")
    assert bench.cpu_threads(8) == 3
    assert bench.cpu_model() is None or isinstance(bench.cpu_model(), str)


def test_official_c_leg():
    """The CPU baseline's second leg: cas.rs's per-file sequence through the BLAKE3 team's C
    library (oracle/ext_b3.c) — its keys equal the oracle's and it reports its library."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    from oracle.pyoracle import ExtBlake3, Oracle
    try:
        ExtBlake3()
    except OSError:
        import pytest
        pytest.skip("no libclang-cpp.so with the BLAKE3 C API in this image")
    rng = np.random.default_rng(3)
    host = rng.integers(0, 256, (64, 57344), dtype=np.uint8)
    hs = rng.integers(102_401, 2 ** 40, 64, dtype=np.uint64)
    gk = Oracle().fast_cas_keys_strided(host.reshape(-1), 57344, 57344, hs, 2)
    leg = bench.official_c_leg(host, hs, gk, 2, 0.1)
    assert leg["parity_vs_gpu"] and leg["value"] > 0 and leg["value_1thread"] > 0
    assert "libclang-cpp.so" in leg["library"] and leg["threads"] == 2
    leg = bench.official_c_leg(host, hs, gk ^ np.uint64(1), 2, 0.05)
    assert not leg["parity_vs_gpu"]


def test_smi_sampler_and_session_evidence(monkeypatch):
    """bench.py's live power sampling picks THIS rank's card by PCI bus (never another card's
    numbers when several are listed and none matches) and tolerates a missing or garbled
    rocm-smi; the VALU / power evidence read from the committed same-session file is marked
    as not measured in the run."""
    import json as _json
    import subprocess
    import time as _time
    import types
    sys.path.insert(0, ROOT)
    import bench
    smi = {"card0": {"PCI Bus": "0000:05:00.0", "Current Socket Graphic Package Power (W)": "1000.0",
                     "sclk clock speed:": "(1900Mhz)"},
           "card1": {"PCI Bus": "0000:f1:00.0", "Current Socket Graphic Package Power (W)": "1361.0",
                     "sclk clock speed:": "(2212Mhz)"}}
    out = {"stdout": _json.dumps(smi)}

    def fake_run(cmd, **kw):
        if out["stdout"] is None:
            raise OSError("no rocm-smi")
        return types.SimpleNamespace(stdout=out["stdout"], returncode=0)
    monkeypatch.setattr(subprocess, "run", fake_run)
    s = bench.SmiSampler(types.SimpleNamespace(pci_bus_id=0xF1), settle_s=0.0)
    _time.sleep(0.6)
    live = s.stop()
    assert live["power_w_median"] == 1361.0 and live["sclk_mhz_median"] == 2212.0 and live["pci_bus"] == 0xF1
    s = bench.SmiSampler(types.SimpleNamespace(pci_bus_id=0x33), settle_s=0.0)  # no such card
    _time.sleep(0.3)
    assert s.stop() is None
    for bad in (None, "not json", "[1, 2]"):
        out["stdout"] = bad
        s = bench.SmiSampler(types.SimpleNamespace(pci_bus_id=0xF1), settle_s=0.0)
        _time.sleep(0.3)
        assert s.stop() is None
    valu, power = bench.valu_power_evidence("sd_cas_sampled_group_kernel", 1310720, 24.0,
                                            {"value": 54e6, "n_gpus": 1}, live)
    assert valu["measured_in_this_run"] is False and valu["session"]
    assert 0.3 < valu["instr_rate_frac_of_peak"] < 0.6 and valu["valu_busy"] > 0.9
    assert power["measured_in_this_run"] is False and power["live"]["measured_in_this_run"] is True
    assert 0.8 < power["live"]["sustained_frac_of_capped_ceiling"] < 1.0
    assert 0.8 < power["session_frac_of_capped_ceiling"] < 1.0
