"""Multi-GPU Object grouping: files sharded by index across ranks, cas keys exchanged by
key range with one all-to-all (RCCL over xGMI on MI355X), grouped locally, and the
representative sent back to each file's owner with the mirror all-to-all.

Reference: the grouping of core/src/object/file_identifier/mod.rs:98-350.
The reference runs on one host thread; here G ranks (one process per GPU) each hash
their contiguous slice of files (no communication), then:

  1. key-range partition of the local keys, dest(k) = floor(k * G / 2^64)
     (BLAKE3 keys are uniform)                                   [HIP: sd_cas_partition_dev]
  2. ONE all_to_all_single of 12-byte rows (key u64, global file idx u32)          [RCCL]
  3. grouping of the received pairs: rep = min global idx over equal keys
                                                                 [HIP: sd_cas_group_min_dev]
  4. mirror all_to_all_single of the u32 reps (4 B/key); scatter to local file order [RCCL]

Every key lives on exactly one rank after step 2, so step 3's minimum is the global one:
rep(f) = min{ g : key(g) == key(f) } over all ranks, the single-GPU contract.

Two forms of step 2:
  * fixed capacity (``capacity=`` given, the production form): every rank sends G blocks of
    `cap` rows + G spill blocks whatever its part sizes are — uniform keys put n/G +- a few
    sqrt(n/G) keys in each part, so no part sizes travel to the host and the step has NO
    host synchronisation (equal-split all_to_all); unused slots carry a sentinel key outside
    the receiver's range.  A part larger than cap + spill (heavily duplicated libraries: the
    copies of one file all go to one rank) raises a device flag; :meth:`ShardResult.resolve`
    (called by ``.objects``) reads it once and redoes the step with the exact form;
  * exact: the part sizes are exchanged first and read on the host for the split lists.

``ops`` supplies the device primitives; in production it is the HIP engine
(:class:`HipShardOps`).  Tests on CPU pass a host implementation to check the exchange
logic with the gloo backend — that is a test double for the kernels, not a fallback.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Protocol

import torch
import torch.distributed as dist


class ShardOps(Protocol):
    def partition(self, keys: torch.Tensor, parts: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """key-range partition -> (part-contiguous keys, their int32 input positions,
        int64 part sizes)"""

    def group_min(self, keys: torch.Tensor, vals: torch.Tensor) -> tuple[torch.Tensor, int]:
        """out[i] = min{ vals[j] : keys[j] == keys[i] } (int32), distinct keys"""

    def group_min_dev(self, keys: torch.Tensor, vals: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """same, the distinct-key count as an int64 [1] device tensor (no host sync)"""

    def pack(self, keys: torch.Tensor, pos: torch.Tensor, file0: int) -> torch.Tensor:
        """int32 rows [n, 3] = (key lo32, key hi32, u32(file0 + pos))"""

    def split(self, rows: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """received rows -> (int64 keys, int32 u32-bit vals)"""

    def unpack(self, back: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
        """int64 rep with rep[pos[j]] = u32(back[j])"""

    def pack_fixed(self, keys, pos, counts, parts: int, cap: int, spill: int, file0: int):
        """(rows [parts*cap, 3], spill rows [parts*spill, 3], overflow int32 [1])"""

    def split_fixed(self, rows, sentinel: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(int64 keys, int32 vals, int64 [1] = number of sentinel rows; row j with key ==
        sentinel gets key sentinel + j)"""

    def unpack_fixed(self, back, spill_back, pos, counts, parts: int, cap: int, spill: int) -> torch.Tensor:
        """int64 rep: mirror of pack_fixed"""


def _cs(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


class HipShardOps:
    """The production ops: libsd_hip_cas.so on the rank's GPU."""

    def __init__(self, eng):
        self.eng = eng
        self.L = eng.L

    def _chk(self, rc: int, what: str) -> None:
        self.eng._check(rc, what)

    def partition(self, keys, parts):
        n = keys.numel()
        ko = torch.empty_like(keys)
        po = torch.empty(n, dtype=torch.int32, device=keys.device)
        counts = torch.empty(parts, dtype=torch.int64, device=keys.device)
        self.eng.partition(keys, parts, ko, po, counts, stream=_cs(keys))
        return ko, po, counts

    def group_min(self, keys, vals):
        out = torch.empty(keys.numel(), dtype=torch.int32, device=keys.device)
        objects = self.eng.group_min(keys, vals, out, stream=_cs(keys))
        return out, objects

    def group_min_dev(self, keys, vals):
        out = torch.empty(keys.numel(), dtype=torch.int32, device=keys.device)
        obj = torch.empty(1, dtype=torch.int64, device=keys.device)
        self.eng.group_min(keys, vals, out, stream=_cs(keys), want_objects=False)
        self._chk(self.L.sd_cas_copy_objects_dev(self.eng.h, obj.data_ptr(), _cs(keys)), "copy_objects")
        return out, obj

    def pack(self, keys, pos, file0):
        rows = torch.empty((keys.numel(), 3), dtype=torch.int32, device=keys.device)
        self.eng.exchange_pack(keys, pos, file0, rows, stream=_cs(keys))
        return rows

    def split(self, rows):
        m = rows.shape[0]
        keys = torch.empty(m, dtype=torch.int64, device=rows.device)
        vals = torch.empty(m, dtype=torch.int32, device=rows.device)
        self.eng.exchange_split(rows, keys, vals, stream=_cs(rows))
        return keys, vals

    def unpack(self, back, pos):
        rep = torch.empty(back.numel(), dtype=torch.int64, device=back.device)
        self.eng.exchange_unpack(back, pos, rep, stream=_cs(back))
        return rep

    def pack_fixed(self, keys, pos, counts, parts, cap, spill, file0):
        dev = keys.device
        rows = torch.empty((parts * cap, 3), dtype=torch.int32, device=dev)
        srows = torch.empty((max(parts * spill, 1), 3), dtype=torch.int32, device=dev)
        overflow = torch.zeros(1, dtype=torch.int32, device=dev)
        self._chk(self.L.sd_cas_exchange_pack_fixed_dev(
            self.eng.h, keys.data_ptr(), pos.data_ptr(), counts.data_ptr(), parts, cap, spill,
            file0, rows.data_ptr(), srows.data_ptr(), overflow.data_ptr(), _cs(keys)), "pack_fixed")
        return rows, srows[:parts * spill], overflow

    def split_fixed(self, rows, sentinel):
        m = rows.shape[0]
        keys = torch.empty(m, dtype=torch.int64, device=rows.device)
        vals = torch.empty(m, dtype=torch.int32, device=rows.device)
        flag = torch.zeros(1, dtype=torch.int64, device=rows.device)
        self._chk(self.L.sd_cas_exchange_split_fixed_dev(
            self.eng.h, rows.data_ptr(), m, sentinel & 0xFFFFFFFFFFFFFFFF, keys.data_ptr(),
            vals.data_ptr(), flag.data_ptr(), _cs(rows)), "split_fixed")
        return keys, vals, flag

    def unpack_fixed(self, back, spill_back, pos, counts, parts, cap, spill):
        n = pos.numel()
        rep = torch.empty(n, dtype=torch.int64, device=pos.device)
        sb = spill_back if spill_back.numel() else back
        self._chk(self.L.sd_cas_exchange_unpack_fixed_dev(
            self.eng.h, back.data_ptr(), sb.data_ptr(), pos.data_ptr(), counts.data_ptr(), parts,
            cap, spill, rep.data_ptr(), _cs(pos)), "unpack_fixed")
        return rep


def range_start(r: int, parts: int) -> int:
    """First key of range r of `parts`: ceil(r * 2^64 / parts) (r = parts wraps to 0)."""
    r %= parts
    return -((-(r << 64)) // parts) if r else 0


def fixed_capacity(n_per_rank: int, parts: int) -> tuple[int, int]:
    """(cap, spill) of the fixed-capacity exchange for ranks holding <= n_per_rank uniform
    keys: the mean part plus 8 standard deviations (binomial), and a spill block of 1/16
    more — overflow then needs > 8 sigma (uniform keys) or heavy duplication."""
    mean = n_per_rank / parts
    sd = math.sqrt(max(mean * (1 - 1 / parts), 1.0))
    cap = int(math.ceil(mean + 8 * sd)) + 64
    return cap, max(256, cap // 16)


@dataclass
class ShardResult:
    """One grouping's result.  ``rep`` and ``objects`` resolve first: with the fixed-capacity
    form an overflowed part leaves garbage in the raw representatives until the exact redo,
    so neither is readable before :meth:`resolve` has run (it runs on first access)."""
    _rep: torch.Tensor       # int64 global idx of the file owning each local file's Object
    objects_dev: torch.Tensor  # int64 [1]: Objects over all ranks (= distinct keys), device
    sent: Optional[int] = None  # keys this rank sent to other ranks (exact form only)
    overflow: Optional[torch.Tensor] = None  # int32 [1] (fixed form): a part exceeded cap+spill
    _redo: Optional[object] = field(default=None, repr=False)

    def resolve(self) -> "ShardResult":
        """Read the overflow flag (one host sync) and, if any rank's part overflowed its fixed
        capacity, redo the grouping with the exact exchange.  Collective: every rank calls it
        (the flag was max-reduced, so all ranks agree)."""
        if self.overflow is not None:
            if int(self.overflow.item()):
                exact = self._redo()
                self._rep, self.objects_dev, self.sent = exact._rep, exact.objects_dev, exact.sent
            self.overflow = None
            self._redo = None
        return self

    @property
    def rep(self) -> torch.Tensor:
        """rep(f) = min global idx of f's key (resolves the overflow flag first: collective)."""
        self.resolve()
        return self._rep

    @property
    def objects(self) -> int:
        self.resolve()
        return int(self.objects_dev.item())


def sharded_group(local_keys: torch.Tensor, file0: int, ops: ShardOps, group=None,
                  capacity: Optional[tuple[int, int]] = None, mark=None) -> ShardResult:
    """Canonical grouping across all ranks: rep(f) = min{ g : key(g) == key(f) }.
    capacity = (cap, spill) selects the sync-free fixed-capacity exchange (every rank must
    pass the same values, e.g. fixed_capacity(max files per rank, world)); None = exact.
    mark(name), if given, is called after each phase of the fixed form (partition, pack,
    all_to_all, group, all_to_all_back, unpack, all_reduce) on the issuing thread — the
    bench records a stream event there to split the exchange's time."""
    if file0 + local_keys.numel() > (1 << 32):
        raise ValueError("sharded_group: global file idx must fit in u32")
    if capacity is None:
        return _sharded_group_exact(local_keys, file0, ops, group)
    return _sharded_group_fixed(local_keys, file0, ops, group, capacity, mark)


def exchange_bytes_per_step(world: int, capacity: tuple[int, int]) -> int:
    """Bytes one rank sends to OTHER ranks per fixed-capacity step: (cap + spill) 12-byte
    rows and the mirror 4-byte reps to each of the world - 1 peers (its own block stays)."""
    cap, spill = capacity
    return (world - 1) * (cap + spill) * (12 + 4)


def _sharded_group_exact(local_keys, file0, ops, group) -> ShardResult:
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = local_keys.device
    n = local_keys.numel()
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
    return ShardResult(_rep=rep, objects_dev=tot, sent=n - int(sc[rank]))


def _sharded_group_fixed(local_keys, file0, ops, group, capacity, mark=None) -> ShardResult:
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:  # one range: no slot can hold a key outside it, nothing to exchange
        return _sharded_group_exact(local_keys, file0, ops, group)
    cap, spill = capacity
    dev = local_keys.device
    mark = mark or (lambda name: None)
    pkeys, ppos, counts = ops.partition(local_keys, world)                    # 1
    mark("partition")
    rows, srows, overflow = ops.pack_fixed(pkeys, ppos, counts, world, cap, spill, file0)
    mark("pack")
    rrows = torch.empty_like(rows)
    dist.all_to_all_single(rrows, rows, group=group)                          # 2: equal splits
    if spill:
        rsrows = torch.empty_like(srows)
        dist.all_to_all_single(rsrows, srows, group=group)
        rrows = torch.cat([rrows, rsrows])
    mark("all_to_all")
    rkeys, ridx, nsent = ops.split_fixed(rrows, range_start(rank + 1, world))
    rep_min, obj = ops.group_min_dev(rkeys, ridx)                             # 3
    tot = obj - nsent                             # each sentinel row is one extra key
    mark("group")
    back = torch.empty(world * cap, dtype=torch.int32, device=dev)
    dist.all_to_all_single(back, rep_min[:world * cap].contiguous(), group=group)   # 4
    sback = torch.empty(world * spill, dtype=torch.int32, device=dev)
    if spill:
        dist.all_to_all_single(sback, rep_min[world * cap:].contiguous(), group=group)
    mark("all_to_all_back")
    rep = ops.unpack_fixed(back, sback, ppos, counts, world, cap, spill)
    mark("unpack")
    dist.all_reduce(tot, group=group)
    dist.all_reduce(overflow, op=dist.ReduceOp.MAX, group=group)
    mark("all_reduce")
    return ShardResult(_rep=rep, objects_dev=tot, overflow=overflow,
                       _redo=lambda: _sharded_group_exact(local_keys, file0, ops, group))
