#!/usr/bin/env python3
"""A/B of the grouping entry points on one batch: group (vals = positions) vs group_min with
a vals array (the exchange's received global indices) vs group_min with vals = None, on the
exchange-shaped input (1.42 M rows, world 8) and on 1.31 M uniform keys.  Times = HIP events
over 20 back-to-back calls (GPU-bound), ms per call."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from spacedrive_amd import CasEngine  # noqa: E402
from spacedrive_amd.shard import HipShardOps, fixed_capacity, range_start  # noqa: E402

eng = CasEngine(0)
ops = HipShardOps(eng)


def per_call(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / reps)
    return best


world, n, rank = 8, 1310720, 3
cap, spill = fixed_capacity(n, world)
rng = np.random.default_rng(2)
pool = rng.integers(0, 2 ** 64, int(n * 0.7), dtype=np.uint64)
keys = torch.from_numpy(pool[rng.integers(0, len(pool), n)].view(np.int64)).cuda()
pk, pp, counts = ops.partition(keys, world)
rows, srows, _ = ops.pack_fixed(pk, pp, counts, world, cap, spill, rank * n)
rk, rv, _ = ops.split_fixed(torch.cat([rows, srows]), range_start(rank + 1, world))
out = {}
rku = rk.cpu().numpy().view(np.uint64)
perm = torch.from_numpy(rng.permutation(rk.numel())).cuda()
real = rv.cpu().numpy().view(np.uint32) != 0xFFFFFFFF
n2 = rk.numel()
more = torch.from_numpy(pool[rng.integers(0, len(pool), n2)].view(np.int64)).cuda()
variants = [("exchange_1.42M", rk, rv), ("exchange_permuted", rk[perm].contiguous(), rv[perm].contiguous()),
            ("exchange_real_rows_only", rk[torch.from_numpy(real).cuda()].contiguous(), None),
            ("uniform_1.42M", more, None), ("uniform_1.31M", keys, None)]
rr = rku[real]
ns = int((~real).sum())
seq = (np.uint64(range_start(rank + 1, world)) + np.arange(ns, dtype=np.uint64))
rnd = rng.integers(0, 2 ** 64, ns, dtype=np.uint64)
variants += [("real_plus_seq_sentinels", torch.from_numpy(np.concatenate([rr, seq]).view(np.int64)).cuda(), None),
             ("real_plus_random", torch.from_numpy(np.concatenate([rr, rnd]).view(np.int64)).cuda(), None),
             ("seq_only", torch.from_numpy(seq.view(np.int64)).cuda(), None),
             ("random_only", torch.from_numpy(rnd.view(np.int64)).cuda(), None)]
if len(sys.argv) > 1:
    variants = [v for v in variants if v[0] in sys.argv[1:]]
for name, k, v in variants:
    m = k.numel()
    o = torch.empty(m, dtype=torch.int32, device="cuda")
    rep = torch.empty(m, dtype=torch.int64, device="cuda")
    vv = v if v is not None else torch.arange(m, dtype=torch.int32, device="cuda")
    out[name] = {
        "group_ms": per_call(lambda: eng.group(k, rep, stream=torch.cuda.current_stream().cuda_stream, want_objects=False)),
        "group_min_vals_ms": per_call(lambda: eng.group_min(k, vv, o, stream=torch.cuda.current_stream().cuda_stream, want_objects=False)),
        "group_min_none_ms": per_call(lambda: eng.group_min(k, None, o, stream=torch.cuda.current_stream().cuda_stream, want_objects=False)),
    }
print(json.dumps(out), flush=True)
