"""Per-block phase timing of sd_part_scatter_mix (instrumented build tools/ablib/ts_scatter.so,
patch tools/ab_patches/ts_scatter.py) at n keys: prologue (totals + scan) and each trip, in us;
blocks resident over time.  Usage: SD_HIP_CAS_LIB=... n"""
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
    eng.group(keys, rep)
torch.cuda.synchronize()
L = _native.lib()
buf = np.zeros(4096 * 8, dtype=np.uint64)
assert L.sd_dbg_scatter_ts(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
ts = buf.reshape(4096, 8).astype(np.int64)
nblk = int((ts[:, 0] > 0).sum())
ts = ts[:nblk]
t0 = ts[:, 0].min()
rel = (ts - t0) * 10  # ns
ntrip = int((ts[:, 2:] > 0).sum(axis=1).max())
last = np.array([rel[i, 1 + int((ts[i, 2:] > 0).sum())] for i in range(nblk)])
out = {"n": n, "blocks": nblk, "trips_max": ntrip, "span_us": float(last.max() / 1e3),
       "prologue_us": {"med": float(np.median(rel[:, 1] - rel[:, 0]) / 1e3), "p90": float(np.percentile(rel[:, 1] - rel[:, 0], 90) / 1e3)}}
for t in range(ntrip):
    d = rel[:, 2 + t] - rel[:, 1 + t]
    m = ts[:, 2 + t] > 0
    out[f"trip{t}_us"] = {"med": float(np.median(d[m]) / 1e3), "p90": float(np.percentile(d[m], 90) / 1e3)}
life = last - rel[:, 0]
out["life_us"] = {"med": float(np.median(life) / 1e3), "p90": float(np.percentile(life, 90) / 1e3)}
grid = np.linspace(0, last.max(), 40)
out["alive_over_time"] = [int(((rel[:, 0] <= t) & (last >= t)).sum()) for t in grid]
print(json.dumps(out), flush=True)
