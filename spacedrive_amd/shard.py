"""Multi-GPU Object grouping: files sharded by index across ranks, cas keys exchanged by
key range with one all-to-all (RCCL over xGMI on MI355X), grouped locally, and the
representative sent back to each file's owner with the mirror all-to-all.

Reference: the grouping of core/src/object/file_identifier/mod.rs:98-350.
The reference runs on one host thread; here G ranks (one process per GPU) each hash
their contiguous slice of files (no communication), then:

  1. local stable sort of (key, local idx)                  [HIP radix sort]
  2. split points of the key ranges dest(k) = floor(k * G / 2^64) on the sorted keys
  3. all_to_all_single of keys and global idx (counts first)   [RCCL]
  4. local stable sort of the received (key, recv position) -> runs -> rep = head's
     global idx (received runs arrive in rank order and each run is idx-ascending, so
     the head of an equal-key run holds the global minimum idx)   [HIP]
  5. mirror all_to_all_single of the reps; scatter into local idx order  [RCCL]

``ops`` supplies the three device primitives; in production it is the HIP engine
(:class:`HipShardOps`).  Tests on CPU pass a host implementation to check the exchange
logic with the gloo backend — that is a test double for the kernels, not a fallback.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Protocol

import torch
import torch.distributed as dist

SIGN = -(1 << 63)  # int64 bit pattern of 0x8000_0000_0000_0000


class ShardOps(Protocol):
    def sort_pairs(self, keys: torch.Tensor, vals: Optional[torch.Tensor]) -> tuple[torch.Tensor, torch.Tensor]:
        """stable sort of u64 keys (int64 storage) -> (sorted keys, int32 vals)"""

    def group_sorted(self, skeys: torch.Tensor, svals: torch.Tensor) -> tuple[torch.Tensor, int]:
        """rep[svals[i]] = svals[head(i)] (int32), objects"""


class HipShardOps:
    """The production ops: libsd_hip_cas.so on the rank's GPU."""

    def __init__(self, eng):
        self.eng = eng

    def sort_pairs(self, keys, vals):
        n = keys.numel()
        ko = torch.empty_like(keys)
        vo = torch.empty(n, dtype=torch.int32, device=keys.device)
        self.eng.sort_pairs(keys, vals, ko, vo, 0, 64, stream=torch.cuda.current_stream().cuda_stream)
        return ko, vo

    def group_sorted(self, skeys, svals):
        rep = torch.empty(skeys.numel(), dtype=torch.int32, device=skeys.device)
        objects = self.eng.group_sorted(skeys, svals, rep,
                                        stream=torch.cuda.current_stream().cuda_stream)
        return rep, objects


def key_range_splits(sorted_keys: torch.Tensor, world: int) -> torch.Tensor:
    """counts[r] = #keys with floor(k * world / 2^64) == r, keys sorted as unsigned u64.

    Flipping the sign bit maps unsigned order onto signed int64 order, so the boundaries
    ceil(r * 2^64 / world) can be located with torch.searchsorted."""
    flipped = sorted_keys ^ SIGN
    bounds = []
    for r in range(1, world):
        b = -((-(r << 64)) // world)  # ceil(r * 2^64 / world), unsigned
        fb = b ^ (1 << 63)            # sign-flipped ...
        bounds.append(fb - (1 << 64) if fb >= (1 << 63) else fb)  # ... as int64
    bt = torch.tensor(bounds, dtype=torch.int64, device=sorted_keys.device)
    pos = torch.searchsorted(flipped, bt)  # number of keys < boundary
    edges = torch.cat([torch.zeros(1, dtype=torch.int64, device=pos.device), pos,
                       torch.tensor([sorted_keys.numel()], dtype=torch.int64, device=pos.device)])
    return edges[1:] - edges[:-1]


@dataclass
class ShardResult:
    rep: torch.Tensor        # int64 global idx of the file owning each local file's Object
    objects: int             # Objects over all ranks (= distinct keys)
    sent: int                # keys this rank sent to other ranks


def sharded_group(local_keys: torch.Tensor, file0: int, ops: ShardOps,
                  group=None) -> ShardResult:
    """Canonical grouping across all ranks: rep(f) = min{ g : key(g) == key(f) }."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = local_keys.device
    n = local_keys.numel()
    skeys, sidx = ops.sort_pairs(local_keys, None)               # 1
    send_counts = key_range_splits(skeys, world)                  # 2
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)  # counts exchange
    sc = send_counts.cpu().tolist()
    rc = recv_counts.cpu().tolist()
    gidx = sidx.to(torch.int64) + file0
    rkeys = torch.empty(sum(rc), dtype=torch.int64, device=dev)
    ridx = torch.empty(sum(rc), dtype=torch.int64, device=dev)
    dist.all_to_all_single(rkeys, skeys, rc, sc, group=group)     # 3
    dist.all_to_all_single(ridx, gidx, rc, sc, group=group)
    m = rkeys.numel()
    if m:
        k2, pos = ops.sort_pairs(rkeys, None)                     # 4
        rep_pos, objects = ops.group_sorted(k2, pos)
        rep_global = ridx[rep_pos.to(torch.int64)]
    else:
        rep_global = torch.empty(0, dtype=torch.int64, device=dev)
        objects = 0
    back = torch.empty(n, dtype=torch.int64, device=dev)
    dist.all_to_all_single(back, rep_global, sc, rc, group=group)  # 5
    rep = torch.empty(n, dtype=torch.int64, device=dev)
    rep[sidx.to(torch.int64)] = back
    tot = torch.tensor([objects], dtype=torch.int64, device=dev)
    dist.all_reduce(tot, group=group)
    return ShardResult(rep=rep, objects=int(tot.item()), sent=n - int(sc[rank]))
