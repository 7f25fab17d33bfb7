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
