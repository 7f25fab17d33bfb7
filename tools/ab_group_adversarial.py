#!/usr/bin/env python3
"""Grouping cost on adversarial key sets at the bench's 1.31M keys (one key making up 40 % of
the library; keys ordered by their bucket), HIP-event medians; checked against numpy."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.pyoracle import np_mix64  # noqa: E402
from spacedrive_amd import CasEngine  # noqa: E402


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
rng = np.random.default_rng(5)
n = 1310720
base = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
hot = base.copy()
hot[rng.random(n) < 0.4] = np.uint64(0xDEADBEEFCAFEF00D)
cases = {"uniform": base, "one key 40 %": hot, "bucket-sorted": base[np.argsort(np_mix64(base))]}
for name, keys in cases.items():
    dk = torch.from_numpy(keys.view(np.int64)).cuda()
    rep = torch.empty(n, dtype=torch.int32, device="cuda")
    eng.group(dk, rep)
    uniq, first, inv = np.unique(keys, return_index=True, return_inverse=True)
    ok = bool((rep.cpu().numpy() == first[inv]).all())
    print(json.dumps({"case": name, "ms": timed(lambda: eng.group(dk, rep, want_objects=False)), "ok": ok}), flush=True)
