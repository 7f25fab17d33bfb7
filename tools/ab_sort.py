#!/usr/bin/env python3
"""LSD radix sort A/B: sd_cas_sort_pairs_dev (64-bit keys, 8 passes) and the sort+runs
grouping at 1.31M and 12.5M keys, HIP-event medians; results checked against numpy."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from spacedrive_amd import CasEngine  # noqa: E402


def timed(fn, reps=5):
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
rng = np.random.default_rng(8)
for n in (1310720, 12500000):
    keys_h = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
    keys = torch.from_numpy(keys_h.view(np.int64)).cuda()
    ko = torch.empty_like(keys)
    vo = torch.empty(n, dtype=torch.int32, device="cuda")
    eng.sort_pairs(keys, None, ko, vo)
    order = np.argsort(keys_h, kind="stable")
    ok = bool((ko.cpu().numpy().view(np.uint64) == keys_h[order]).all() and (vo.cpu().numpy() == order).all())
    t = timed(lambda: eng.sort_pairs(keys, None, ko, vo))
    print(json.dumps({"n": n, "sort_ms": t, "gkeys_per_s": n / t / 1e6, "ok": ok}), flush=True)
