#!/usr/bin/env python3
"""GPU-side cost of one step of the N > 1 grouping on one rank (bench shape: 1,310,720 keys
per rank, world 8), without the RCCL transfer.  The all_to_all is emulated in one process:
8 senders each partition + pack their own 1.31 M keys, and receiver `rank` takes block
`rank` (main + spill) of every sender — the rows it would receive.  Timed alone (HIP
events, medians): range partition, fixed-capacity pack, split, group_min of the ~1.42 M
received rows, unpack, and the chain; plus group_min with the padding rows left on ONE
sentinel key (the pre-spread split) for comparison."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from spacedrive_amd import CasEngine  # noqa: E402
from spacedrive_amd.shard import HipShardOps, fixed_capacity, range_start  # noqa: E402


def timed(fn, reps=7):
    fn()
    torch.cuda.synchronize()
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
pool = rng.integers(0, 2 ** 64, int(world * n * 0.7), dtype=np.uint64)
senders = []
for r in range(world):
    k = torch.from_numpy(pool[rng.integers(0, len(pool), n)].view(np.int64)).cuda()
    pk, pp, cnt = ops.partition(k, world)
    rows, srows, ovf = ops.pack_fixed(pk, pp, cnt, world, cap, spill, r * n)
    senders.append((k, pk, pp, cnt, rows.view(world, cap, 3), srows.view(world, spill, 3)))
recv = torch.cat([s[4][rank] for s in senders] + [s[5][rank] for s in senders])
sent = range_start(rank + 1, world)
rk, rv, nsent = ops.split_fixed(recv, sent)
rep_min, obj = ops.group_min_dev(rk, rv)
torch.cuda.synchronize()
pad = rv == -1
hot = torch.where(pad, torch.tensor(sent - 2 ** 64 if sent >= 2 ** 63 else sent, dtype=torch.int64, device="cuda"), rk)
k0, pk0, pp0, cnt0 = senders[rank][:4]
back = rep_min[:world * cap].contiguous()
sback = rep_min[world * cap:].contiguous()
out = {"world": world, "keys": n, "capacity_per_peer": cap, "spill_per_peer": spill,
       "rows_received": int(recv.shape[0]), "padding_rows": int(nsent.item()),
       "partition_ms": timed(lambda: ops.partition(k0, world)),
       "pack_fixed_ms": timed(lambda: ops.pack_fixed(pk0, pp0, cnt0, world, cap, spill, rank * n)),
       "split_fixed_ms": timed(lambda: ops.split_fixed(recv, sent)),
       "group_min_ms": timed(lambda: ops.group_min_dev(rk, rv)),
       "group_min_one_sentinel_key_ms": timed(lambda: ops.group_min_dev(hot, rv)),
       "unpack_fixed_ms": timed(lambda: ops.unpack_fixed(back, sback, pp0, cnt0, world, cap, spill))}


def chain():
    a, b, c = ops.partition(k0, world)
    ops.pack_fixed(a, b, c, world, cap, spill, rank * n)
    kk, vv, f = ops.split_fixed(recv, sent)
    m, ob = ops.group_min_dev(kk, vv)
    ops.unpack_fixed(m[:world * cap].contiguous(), m[world * cap:].contiguous(), b, c, world, cap, spill)


out["chain_ms"] = timed(chain)
print(json.dumps(out), flush=True)
