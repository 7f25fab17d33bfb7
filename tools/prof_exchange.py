#!/usr/bin/env python3
"""GPU-side cost of one step of the N > 1 grouping on one rank (bench shape: 1,310,720 keys
per rank, world 8), without the RCCL transfer: range partition, fixed-capacity pack, split of
the received rows (this rank's own packed rows stand in for the peers'), group_min of ~1.42M
rows incl. sentinels, fixed unpack — each timed alone (HIP events) and the chain."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from spacedrive_amd import CasEngine  # noqa: E402
from spacedrive_amd.shard import HipShardOps, fixed_capacity, range_start  # noqa: E402


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
ops = HipShardOps(eng)
world, n, rank = 8, 1310720, 3
cap, spill = fixed_capacity(n, world)
rng = np.random.default_rng(2)
pool = rng.integers(0, 2 ** 64, int(n * 0.7), dtype=np.uint64)
keys = torch.from_numpy(pool[rng.integers(0, len(pool), n)].view(np.int64)).cuda()
pk, pp, counts = ops.partition(keys, world)
rows, srows, ovf = ops.pack_fixed(pk, pp, counts, world, cap, spill, rank * n)
recv = torch.cat([rows, srows])
rk, rv, flag = ops.split_fixed(recv, range_start(rank + 1, world))
rep_min, obj = ops.group_min_dev(rk, rv)
torch.cuda.synchronize()
out = {"world": world, "keys": n, "capacity_per_peer": cap, "spill_per_peer": spill, "rows_received": int(recv.shape[0]),
       "partition_ms": timed(lambda: ops.partition(keys, world)),
       "pack_fixed_ms": timed(lambda: ops.pack_fixed(pk, pp, counts, world, cap, spill, rank * n)),
       "split_fixed_ms": timed(lambda: ops.split_fixed(recv, range_start(rank + 1, world))),
       "group_min_ms": timed(lambda: ops.group_min_dev(rk, rv)),
       "unpack_fixed_ms": timed(lambda: ops.unpack_fixed(rep_min[:world * cap].contiguous(), rep_min[world * cap:].contiguous(), pp, counts, world, cap, spill))}


def chain():
    a, b, c = ops.partition(keys, world)
    r, s, o = ops.pack_fixed(a, b, c, world, cap, spill, rank * n)
    kk, vv, f = ops.split_fixed(torch.cat([r, s]), range_start(rank + 1, world))
    m, ob = ops.group_min_dev(kk, vv)
    ops.unpack_fixed(m[:world * cap].contiguous(), m[world * cap:].contiguous(), b, c, world, cap, spill)


out["chain_ms"] = timed(chain)
print(json.dumps(out), flush=True)
