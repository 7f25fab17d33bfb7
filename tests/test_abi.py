"""CPU tests of the drop-in boundary: the C-ABI library builds for gfx950, loads, exports
every symbol include/sd_hip_cas.h declares, and refuses to run without a gfx950 device
(no silent CPU fallback).  No compute calls are made here."""
import ctypes
import os
import re

import pytest

from spacedrive_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "sd_hip_cas.h")) as fh:
        text = fh.read()
    return sorted(set(re.findall(r"\b(sd_cas_\w+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    syms = header_symbols()
    for s in ["sd_cas_generate_cas_ids", "sd_cas_group_dev", "sd_cas_file_checksum",
              "sd_cas_hash_sampled_dev", "sd_cas_hash_packed_dev", "sd_cas_ctx_create"]:
        assert s in syms


def test_library_exports_every_header_symbol():
    L = _native.lib()
    missing = [s for s in header_symbols() if not hasattr(L, s)]
    assert not missing, missing
    # and the ctypes signature table covers the header exactly
    assert sorted(n for n, _, _ in _native.SIGNATURES) == header_symbols()


def test_library_is_gfx950_code_object():
    # the fat binary must carry a gfx950 code object
    with open(_native.LIB_PATH, "rb") as fh:
        blob = fh.read()
    assert b"gfx950" in blob


def test_abi_version_and_hex():
    L = _native.lib()
    assert L.sd_cas_abi_version() == 1
    out = ctypes.create_string_buffer(17)
    L.sd_cas_key_to_hex(0xAF1349B9F5F9A1A6, out)
    assert out.value == b"af1349b9f5f9a1a6"


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from spacedrive_amd import CasEngine, CasError
    with pytest.raises(CasError):
        CasEngine(0)


def test_null_context_rejected():
    L = _native.lib()
    assert L.sd_cas_generate_cas_ids(None, None, None, None, 0, None) == -1
    assert L.sd_cas_group_dev(None, None, 0, None, None, None) == -1


def test_one_hip_runtime_per_process():
    """Loading the library before torch must not map a second HIP/HSA runtime (torch ships
    its own libamdhip64.so.7; two runtimes in one process leave the second without a GPU)."""
    import subprocess
    import sys
    code = ("import re, spacedrive_amd._native as n; n.lib(); import torch; "
            "m = open('/proc/self/maps').read(); "
            "print(len(set(re.findall(r'/\\S*libamdhip64\\S*', m))), "
            "len(set(re.findall(r'/\\S*libhsa-runtime64\\S*', m))))")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["1", "1"], out.stdout
