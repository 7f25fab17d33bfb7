"""Grouping A/B driver: the standalone chain (sd_cas_group_dev) on device-generated keys with
30 % duplicates at the given sizes, 10 calls back to back per timing (HIP events), 5 timings;
prints per size the median ms, the HBM fraction at the chain's algorithmic bytes and a rep
digest (variants must agree).  The library comes from SD_HIP_CAS_LIB (tools/ab_run style)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spacedrive_amd import CasEngine  # noqa: E402

eng = CasEngine(0)
out = {"lib": os.path.basename(os.environ.get("SD_HIP_CAS_LIB", "current"))}
for n in [int(x) for x in (sys.argv[1:] or ["1310720", "12500000"])]:
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    nd = int(n * 0.3)
    base = torch.randint(-2 ** 63, 2 ** 63 - 1, (n - nd,), dtype=torch.int64, device="cuda", generator=g)
    keys = torch.cat([base, base[torch.randint(0, n - nd, (nd,), device="cuda", generator=g)]])
    keys = keys[torch.randperm(n, device="cuda", generator=g)]
    rep = torch.empty(n, dtype=torch.int32, device="cuda")
    obj = eng.group(keys, rep)
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            eng.group(keys, rep, want_objects=False)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / 10)
    ms = float(np.median(ts))
    bpk = 36 if n <= 256 * 5632 else (68 if n <= 40_000_000 else 76)
    r = rep.cpu().numpy().astype(np.uint64)
    out[str(n)] = {"ms": ms, "all": ts, "objects": obj, "hbm_frac": n * bpk / (ms / 1e3) / 8e12,
                   "rep_digest": f"{int((r * 0x9E3779B97F4A7C15).sum() & 0xFFFFFFFFFFFFFFFF):016x}"}
    del keys, rep, base
    torch.cuda.empty_cache()
print(json.dumps(out), flush=True)
