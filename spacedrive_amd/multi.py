"""Single-process multi-device engine (C ABI sd_cas_multi_*): the form the Rust core uses
to drive every local MI355X from one process.  Shards = contiguous file ranges, one
context each; the grouping exchange is peer copies over xGMI (see sd_multi.cpp).
The multi-PROCESS form (one rank per GPU, RCCL all-to-all) is spacedrive_amd/shard.py."""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _native
from ._native import CasError
from .cas import _sizes_u64


class MultiEngine:
    def __init__(self, devices: Sequence[int]):
        self.L = _native.lib()
        self.devices = list(devices)
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        rc = self.L.sd_cas_multi_create(arr, len(self.devices), ctypes.byref(h))
        if rc != 0:
            why = self.L.sd_cas_multi_last_error(None)
            raise CasError(rc, f"sd_cas_multi_create({self.devices}) failed: "
                               f"{why.decode() if why else ''}")
        self.h = h

    def close(self) -> None:
        if getattr(self, "h", None):
            self.L.sd_cas_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            msg = self.L.sd_cas_multi_last_error(self.h)
            raise CasError(rc, f"{what}: {msg.decode() if msg else ''}")

    def group(self, keys: Sequence, file0: Sequence[int]):
        """keys[i]: int64 torch tensor on devices[i]; returns (reps, objects) with reps[i] an
        int64 tensor of global file idx per key of shard i."""
        import torch
        G = len(self.devices)
        assert len(keys) == G == len(file0)
        reps = [torch.empty(k.numel(), dtype=torch.int64, device=k.device) for k in keys]
        torch.cuda.synchronize()
        kp = (ctypes.c_void_p * G)(*[k.data_ptr() for k in keys])
        rp = (ctypes.c_void_p * G)(*[r.data_ptr() for r in reps])
        ns = (ctypes.c_size_t * G)(*[k.numel() for k in keys])
        f0 = (ctypes.c_uint64 * G)(*[int(f) for f in file0])
        obj = ctypes.c_uint64(0)
        self._check(self.L.sd_cas_multi_group(self.h, kp, ns, f0, rp, ctypes.byref(obj)), "multi_group")
        return reps, int(obj.value)

    def hash_group_sampled_host(self, content: np.ndarray, sizes: np.ndarray, stride: int = 57344):
        n = len(sizes)
        sz = _sizes_u64(sizes)
        keys = np.zeros(n, dtype=np.uint64)
        rep = np.zeros(n, dtype=np.uint64)
        obj = ctypes.c_uint64(0)
        self._check(self.L.sd_cas_multi_hash_group_sampled_host(
            self.h, int(content.ctypes.data), int(stride), int(sz.ctypes.data), n,
            int(keys.ctypes.data), int(rep.ctypes.data), ctypes.byref(obj)), "multi_hash_group")
        return keys, rep, int(obj.value)
