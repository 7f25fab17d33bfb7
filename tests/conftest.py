import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; parity tests proper")


@pytest.fixture(scope="session")
def oracle():
    """The CPU oracle (test infrastructure; oracle/liboracle_cas.so, built on demand)."""
    from oracle.pyoracle import Oracle, build_oracle
    build_oracle()
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def eng():
    """The product engine on cuda:0 — fails loudly when the HIP library or GPU is missing."""
    import torch
    from spacedrive_amd import CasEngine
    assert torch.cuda.is_available(), "GPU tests need a gfx950 device"
    torch.cuda.init()
    return CasEngine(0)


@pytest.fixture(autouse=True)
def _debug_invariants(request):
    """With SD_CAS_DEBUG_INVARIANTS=1 (and SD_HIP_CAS_LIB = libsd_hip_cas_debug.so, the build
    with the device-side conservation checks of csrc/sd_debug.h; tools/gpu_r3_debug.sh), a
    GPU test after which the library's violation counter moved fails, naming the test."""
    if not os.environ.get("SD_CAS_DEBUG_INVARIANTS") or request.node.get_closest_marker("gpu") is None:
        yield
        return
    import ctypes

    from spacedrive_amd import _native
    L = _native.lib()
    fn = L.sd_cas_debug_violations  # AttributeError: not the debug library
    fn.restype = ctypes.c_uint64
    fn.argtypes = []
    before = fn()
    yield
    after = fn()
    assert after == before, f"{after - before} device invariant violation(s) (see the test's stdout)"
