#!/usr/bin/env python3
"""K2 A/B: the packed path (length sort + sd_cas_packed_kernel) on config 2's 1M ragged
whole files and on 500K uniform 57,344-B contents; one JSON line with HIP-event medians and
an xor digest of the keys so builds can be checked against each other."""
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


def digest(k):
    return int(np.bitwise_xor.reduce(k.cpu().numpy().view(np.uint64)))


eng = CasEngine(0)
out = {}
m = 1_000_000
sz = torch.empty(m, dtype=torch.int64, device="cuda")
ln = torch.empty(m, dtype=torch.int32, device="cuda")
of = torch.empty(m, dtype=torch.int64, device="cuda")
nb = eng.synth_small(11, 0, m, sz, ln, of, None)
arena = torch.empty(nb + 64, dtype=torch.uint8, device="cuda")
eng.synth_small(11, 0, m, sz, ln, of, arena)
k = torch.empty(m, dtype=torch.int64, device="cuda")
eng.hash_packed(arena, of, ln, sz, k)
torch.cuda.synchronize()
out["ragged_1m_ms"] = timed(lambda: eng.hash_packed(arena, of, ln, sz, k))
out["ragged_digest"] = digest(k)
out["ragged_gb"] = nb / 1e9
del arena
torch.cuda.empty_cache()
n = int(os.environ.get("AB_UNIFORM_N", "500000"))
content = torch.empty((n, 57344), dtype=torch.uint8, device="cuda")
sizes = torch.empty(n, dtype=torch.int64, device="cuda")
keys = torch.empty(n, dtype=torch.int64, device="cuda")
eng.synth_sampled(3, 0, n, content, sizes, 57344)
offs = torch.arange(n, dtype=torch.int64, device="cuda") * 57344
lens = torch.full((n,), 57344, dtype=torch.int32, device="cuda")
eng.hash_packed(content, offs, lens, sizes, keys)
torch.cuda.synchronize()
out["uniform_ms"] = timed(lambda: eng.hash_packed(content, offs, lens, sizes, keys))
out["uniform_digest"] = digest(keys)
out["uniform_n"] = n
k1 = torch.empty_like(keys)
eng.hash_sampled(content, sizes, k1)
torch.cuda.synchronize()
assert torch.equal(k1, keys)
out["k1_uniform_ms"] = timed(lambda: eng.hash_sampled(content, sizes, k1))
print(json.dumps(out), flush=True)
