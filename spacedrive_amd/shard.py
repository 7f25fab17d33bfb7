"""Multi-GPU Object grouping: files sharded by index across ranks, cas keys exchanged by
key range with one all-to-all (RCCL over xGMI on MI355X), grouped locally, and the
representative sent back to each file's owner with the mirror all-to-all.

Reference: the grouping of core/src/object/file_identifier/mod.rs:98-350.
The reference runs on one host thread; here G ranks (one process per GPU) each hash
their contiguous slice of files (no communication), then:

  1. key-range partition of the local keys, dest(k) = floor(k * G / 2^64)
     (BLAKE3 keys are uniform)                                   [HIP: sd_cas_partition_dev]
  2. all_to_all_single of the part sizes, then ONE all_to_all_single of 12-byte rows
     (key u64, global file idx u32) — 12 B/key instead of two int64 exchanges' 16  [RCCL]
  3. grouping of the received pairs: rep = min global idx over equal keys
                                                                 [HIP: sd_cas_group_min_dev]
  4. mirror all_to_all_single of the u32 reps (4 B/key); scatter to local file order [RCCL]

Every key lives on exactly one rank after step 2, so step 3's minimum is the global one:
rep(f) = min{ g : key(g) == key(f) } over all ranks, the single-GPU contract.

``ops`` supplies the device primitives; in production it is the HIP engine
(:class:`HipShardOps`).  Tests on CPU pass a host implementation to check the exchange
logic with the gloo backend — that is a test double for the kernels, not a fallback.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Protocol

import torch
import torch.distributed as dist


class ShardOps(Protocol):
    def partition(self, keys: torch.Tensor, parts: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """key-range partition -> (part-contiguous keys, their int32 input positions,
        int64 part sizes)"""

    def group_min(self, keys: torch.Tensor, vals: torch.Tensor) -> tuple[torch.Tensor, int]:
        """out[i] = min{ vals[j] : keys[j] == keys[i] } (int32), distinct keys"""

    def pack(self, keys: torch.Tensor, pos: torch.Tensor, file0: int) -> torch.Tensor:
        """int32 rows [n, 3] = (key lo32, key hi32, u32(file0 + pos))"""

    def split(self, rows: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """received rows -> (int64 keys, int32 u32-bit vals)"""

    def unpack(self, back: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
        """int64 rep with rep[pos[j]] = u32(back[j])"""


class HipShardOps:
    """The production ops: libsd_hip_cas.so on the rank's GPU."""

    def __init__(self, eng):
        self.eng = eng

    def partition(self, keys, parts):
        n = keys.numel()
        ko = torch.empty_like(keys)
        po = torch.empty(n, dtype=torch.int32, device=keys.device)
        counts = torch.empty(parts, dtype=torch.int64, device=keys.device)
        self.eng.partition(keys, parts, ko, po, counts,
                           stream=torch.cuda.current_stream().cuda_stream)
        return ko, po, counts

    def group_min(self, keys, vals):
        out = torch.empty(keys.numel(), dtype=torch.int32, device=keys.device)
        objects = self.eng.group_min(keys, vals, out, stream=torch.cuda.current_stream().cuda_stream)
        return out, objects

    def pack(self, keys, pos, file0):
        rows = torch.empty((keys.numel(), 3), dtype=torch.int32, device=keys.device)
        self.eng.exchange_pack(keys, pos, file0, rows, stream=torch.cuda.current_stream().cuda_stream)
        return rows

    def split(self, rows):
        m = rows.shape[0]
        keys = torch.empty(m, dtype=torch.int64, device=rows.device)
        vals = torch.empty(m, dtype=torch.int32, device=rows.device)
        self.eng.exchange_split(rows, keys, vals, stream=torch.cuda.current_stream().cuda_stream)
        return keys, vals

    def unpack(self, back, pos):
        rep = torch.empty(back.numel(), dtype=torch.int64, device=back.device)
        self.eng.exchange_unpack(back, pos, rep, stream=torch.cuda.current_stream().cuda_stream)
        return rep


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
    if file0 + n > (1 << 32):
        raise ValueError("sharded_group: global file idx must fit in u32")
    pkeys, ppos, send_counts = ops.partition(local_keys, world)     # 1
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)  # 2: sizes
    sc = send_counts.cpu().tolist()
    rc = recv_counts.cpu().tolist()
    rows = ops.pack(pkeys, ppos, file0)  # int32 [n, 3]: key lo, key hi, u32 global idx
    m = sum(rc)
    rrows = torch.empty((m, 3), dtype=torch.int32, device=dev)
    dist.all_to_all_single(rrows, rows, rc, sc, group=group)        # 2: (key, idx) rows
    if m:
        rkeys, ridx = ops.split(rrows)
        rep_min, objects = ops.group_min(rkeys, ridx)              # 3: u32 bits in int32
    else:
        rep_min = torch.empty(0, dtype=torch.int32, device=dev)
        objects = 0
    back = torch.empty(n, dtype=torch.int32, device=dev)
    dist.all_to_all_single(back, rep_min, sc, rc, group=group)      # 4
    rep = ops.unpack(back, ppos)
    tot = torch.tensor([objects], dtype=torch.int64, device=dev)
    dist.all_reduce(tot, group=group)
    return ShardResult(rep=rep, objects=int(tot.item()), sent=n - int(sc[rank]))
