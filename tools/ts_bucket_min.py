"""Per-workgroup phase timing of sd_bucket_min (instrumented build tools/ablib/ts_*.so, patch
tools/ab_patches/ts_bucket_min.py): groups n keys (30 % duplicates) a few times, reads the
last call's timestamps (s_memrealtime, 100 MHz) and prints per-phase medians / p90, the
kernel span, and how many workgroups were resident over time.  Usage: SD_HIP_CAS_LIB=... n"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spacedrive_amd import CasEngine, _native  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
eng = CasEngine(0)
g = torch.Generator(device="cuda")
g.manual_seed(5)
nd = int(n * 0.3)
base = torch.randint(-2 ** 63, 2 ** 63 - 1, (n - nd,), dtype=torch.int64, device="cuda", generator=g)
keys = torch.cat([base, base[torch.randint(0, n - nd, (nd,), device="cuda", generator=g)]])
keys = keys[torch.randperm(n, device="cuda", generator=g)]
rep = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(3):
    obj = eng.group(keys, rep)
torch.cuda.synchronize()
L = _native.lib()
nb = 1
while nb * 1536 < n:
    nb *= 2
if n <= 256 * 5632:  # the big tables: 256 coarse buckets (instrumented build ts_big)
    nb = 256
buf = np.zeros(65536 * 5, dtype=np.uint64)
assert L.sd_dbg_bucket_ts(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
ts = buf[: nb * 5].reshape(nb, 5).astype(np.int64)
t0 = ts[:, 0].min()
rel = (ts - t0) * 10  # ns
d = np.diff(rel, axis=1)
out = {"n": n, "buckets": nb, "objects": obj, "span_us": float((rel[:, 4].max()) / 1e3)}
for i, name in enumerate(["bounds_load", "init_keys_barrier", "insert", "lookup_store"]):
    out[name] = {"med_us": float(np.median(d[:, i]) / 1e3), "p90_us": float(np.percentile(d[:, i], 90) / 1e3),
                 "mean_us": float(d[:, i].mean() / 1e3)}
life = rel[:, 4] - rel[:, 0]
out["life"] = {"med_us": float(np.median(life) / 1e3), "p90_us": float(np.percentile(life, 90) / 1e3)}
# residency: workgroups alive at 50 evenly spaced instants
grid = np.linspace(0, rel[:, 4].max(), 50)
alive = [int(((rel[:, 0] <= t) & (rel[:, 4] >= t)).sum()) for t in grid]
out["alive_over_time"] = alive
starts = np.sort(rel[:, 0]) / 1e3
out["start_us_pct"] = {str(p): float(np.percentile(starts, p)) for p in (0, 10, 50, 90, 100)}
print(json.dumps(out), flush=True)
