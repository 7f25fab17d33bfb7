"""Per-block phase timing of sd_region_partition (instrumented build tools/ablib/ts_rpart.so,
patch tools/ab_patches/ts_region_part.py) at n keys (30 % duplicates), in us from the first
block's entry: entry, loaded, histogram, reserved, staged, stored.  Usage: SD_HIP_CAS_LIB=... n"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spacedrive_amd import CasEngine, _native  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_310_720
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
assert L.sd_dbg_rpart_ts(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
ts = buf.reshape(4096, 8).astype(np.int64)
nblk = int((ts[:, 0] > 0).sum())
rel = (ts[:nblk, :6] - ts[:nblk, 0].min()) * 10 / 1e3  # us
names = ["entry", "loaded", "histogram", "reserved", "staged", "stored"]
out = {"n": n, "blocks": nblk, "span_us": float(rel[:, 5].max())}
for i, nm in enumerate(names):
    out[nm] = {"med": round(float(np.median(rel[:, i])), 2), "max": round(float(rel[:, i].max()), 2)}
for i in range(1, 6):
    d = rel[:, i] - rel[:, i - 1]
    out[f"d_{names[i]}"] = {"med": round(float(np.median(d)), 2), "p90": round(float(np.percentile(d, 90)), 2)}
print(json.dumps(out), flush=True)
