#!/usr/bin/env python3
"""cas_id string batches on the device: keys_to_hex and thumbnail path records for 10M keys,
HIP-event medians; bytes written / time."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from spacedrive_amd import CasEngine, thumbnail_dir  # noqa: E402


def timed(fn, reps=7):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


eng = CasEngine(0)
n = 10_000_000
keys = torch.randint(-2 ** 63, 2 ** 63 - 1, (n,), dtype=torch.int64, device="cuda")
hexes = torch.empty(16 * n, dtype=torch.uint8, device="cuda")
t = timed(lambda: eng.keys_to_hex(keys, hexes))
print(json.dumps({"op": "keys_to_hex", "keys": n, "ms": t, "gb_per_s": n * 24 / t / 1e6}), flush=True)
prefix = thumbnail_dir("/home/user/.local/share/spacedrive", "8c3c4fb3-7e2b-4d7e-9f0a-1b2c3d4e5f60")
stride = 128
out = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
t = timed(lambda: eng.thumbnail_paths(keys, prefix, stride, out))
print(json.dumps({"op": "thumbnail_paths", "keys": n, "stride": stride, "prefix_len": len(prefix), "ms": t,
                  "gb_per_s": n * (8 + stride) / t / 1e6}), flush=True)
t = timed(lambda: out.fill_(0))
print(json.dumps({"op": "torch fill_ (same buffer)", "bytes": n * stride, "ms": t, "gb_per_s": n * stride / t / 1e6}), flush=True)
src = torch.empty_like(out)
t = timed(lambda: out.copy_(src))
print(json.dumps({"op": "torch copy_ (same size)", "bytes": n * stride, "ms": t, "gb_per_s": 2 * n * stride / t / 1e6}), flush=True)
