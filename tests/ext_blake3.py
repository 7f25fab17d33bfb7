"""An independent BLAKE3 in this image, for the parity tests (test infrastructure only).

The reference hashes with the external `blake3` 1.5.0 crate (Cargo.lock:1127-1139), which is not
vendored.  The BLAKE3 team's own C implementation (the `c/` directory of the BLAKE3 repository,
version 1.8.2: portable + SSE4.1/AVX2/AVX-512 back ends, the same tree and chunk logic the
crate's C back end follows) is vendored into LLVM (llvm/lib/Support/BLAKE3) under an `llvm_`
prefix, and ROCm's `libclang-cpp.so` exports its C API:
    llvm_blake3_hasher_init / _init_keyed / _init_derive_key / _update / _finalize / _version.
Neither the oracle nor the product links it; the tests compare both against it — the oracle
at every tree shape up to GiB inputs, and the product's kernels directly on the device's
output — so the BLAKE3 arithmetic of every path is pinned by an implementation written by
the algorithm's authors rather than by the oracle's own formulations agreeing.

Nothing here is shipped: the product never loads this module or the library.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

LIB = "/opt/rocm/lib/llvm/lib/libclang-cpp.so"
_HASHER_BYTES = 4096  # sizeof(llvm_blake3_hasher) is 1,912 (key, chunk state, 55-deep CV stack)
_L = None


def _lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            return None
        L = ctypes.CDLL(LIB)  # RTLD_LOCAL: nothing of it joins the global symbol scope
        L.llvm_blake3_version.restype = ctypes.c_char_p
        L.llvm_blake3_hasher_init.argtypes = [ctypes.c_void_p]
        L.llvm_blake3_hasher_init_keyed.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.llvm_blake3_hasher_init_derive_key.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.llvm_blake3_hasher_update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.llvm_blake3_hasher_finalize.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        _L = L
    return _L


def available() -> bool:
    return _lib() is not None


def version() -> str:
    return _lib().llvm_blake3_version().decode()


def _update(L, h, data) -> None:
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        # pieces of 256 MiB: the hasher is incremental, the split changes nothing
        step = 1 << 28
        for off in range(0, a.size, step):
            piece = a[off:off + step]
            L.llvm_blake3_hasher_update(h, piece.ctypes.data, piece.size)
    else:
        b = bytes(data)
        L.llvm_blake3_hasher_update(h, b, len(b))


def _finalize(L, h, out_len: int) -> bytes:
    out = ctypes.create_string_buffer(out_len)
    L.llvm_blake3_hasher_finalize(h, out, out_len)
    return out.raw


def blake3(*pieces, out_len: int = 32) -> bytes:
    """blake3::hash of the concatenation of `pieces` (bytes-like or uint8 arrays)."""
    L = _lib()
    h = ctypes.create_string_buffer(_HASHER_BYTES)
    L.llvm_blake3_hasher_init(h)
    for p in pieces:
        _update(L, h, p)
    return _finalize(L, h, out_len)


def keyed_hash(key: bytes, data) -> bytes:
    assert len(key) == 32
    L = _lib()
    h = ctypes.create_string_buffer(_HASHER_BYTES)
    L.llvm_blake3_hasher_init_keyed(h, key)
    _update(L, h, data)
    return _finalize(L, h, 32)


def derive_key(context: str, material: bytes) -> bytes:
    L = _lib()
    h = ctypes.create_string_buffer(_HASHER_BYTES)
    L.llvm_blake3_hasher_init_derive_key(h, context.encode())
    _update(L, h, material)
    return _finalize(L, h, 32)


def cas_key(content, size: int) -> int:
    """The cas key of cas.rs:23-62: big-endian u64 of BLAKE3(le64(size) || content)[0..8]."""
    return int.from_bytes(blake3(int(size).to_bytes(8, "little"), content)[:8], "big")
