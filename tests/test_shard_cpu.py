"""CPU (gloo) tests of the multi-GPU grouping exchange in spacedrive_amd/shard.py.

The device primitives (radix sort, run grouping) are replaced by a host test double so
the key-range partition, the two all-to-alls and the scatter-back can be checked with
world_size 2 and 4 on the CPU.  The double is test-only; production uses HipShardOps.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def range_part(k: np.ndarray, parts: int) -> np.ndarray:
    """floor(k * parts / 2^64) for u64 k, exactly (the contract of sd_cas_partition_dev)."""
    hi, lo = k >> np.uint64(32), k & np.uint64(0xFFFFFFFF)
    t = hi * np.uint64(parts) + ((lo * np.uint64(parts)) >> np.uint64(32))
    return (t >> np.uint64(32)).astype(np.int64)


class HostOps:
    """Test double of HipShardOps (numpy), same contracts: the partition's order inside a
    part is unspecified, so the double scrambles it to keep the exchange honest."""

    def __init__(self, seed: int = 0):
        self.rng = np.random.default_rng(seed)

    def partition(self, keys, parts):
        k = keys.numpy().view(np.uint64)
        d = range_part(k, parts)
        order = np.lexsort((self.rng.random(len(k)), d))  # part-contiguous, scrambled inside
        counts = np.bincount(d, minlength=parts).astype(np.int64)
        return (torch.from_numpy(k[order].view(np.int64).copy()),
                torch.from_numpy(order.astype(np.int32)), torch.from_numpy(counts))

    def group_min(self, keys, vals):
        k = keys.numpy()
        v = vals.numpy().view(np.uint32)
        uniq, inv = np.unique(k, return_inverse=True)
        mins = np.full(len(uniq), 0xFFFFFFFF, dtype=np.uint32)
        np.minimum.at(mins, inv, v)
        return torch.from_numpy(mins[inv].view(np.int32).copy()), len(uniq)

    # the row contracts of sd_cas_exchange_{pack,split,unpack}_dev
    def pack(self, keys, pos, file0):
        k = keys.numpy().view(np.uint64)
        rows = np.empty((len(k), 3), dtype=np.uint32)
        rows[:, 0] = k & 0xFFFFFFFF
        rows[:, 1] = k >> np.uint64(32)
        rows[:, 2] = (pos.numpy().astype(np.uint64) + np.uint64(file0)) & 0xFFFFFFFF
        return torch.from_numpy(rows.view(np.int32))

    def split(self, rows):
        r = rows.numpy().view(np.uint32)
        k = r[:, 0].astype(np.uint64) | (r[:, 1].astype(np.uint64) << np.uint64(32))
        return torch.from_numpy(k.view(np.int64).copy()), torch.from_numpy(r[:, 2].view(np.int32).copy())

    def unpack(self, back, pos):
        rep = np.empty(len(back), dtype=np.int64)
        rep[pos.numpy()] = back.numpy().view(np.uint32)
        return torch.from_numpy(rep)

    def group_min_dev(self, keys, vals):
        out, objects = self.group_min(keys, vals)
        return out, torch.tensor([objects], dtype=torch.int64)

    # the contracts of sd_cas_exchange_{pack,split,unpack}_fixed_dev
    def pack_fixed(self, keys, pos, counts, parts, cap, spill, file0):
        from spacedrive_amd.shard import range_start
        k = keys.numpy().view(np.uint64)
        p = pos.numpy().astype(np.uint64)
        c = counts.numpy()
        off = np.concatenate([[0], np.cumsum(c)[:-1]])
        rows = np.empty((parts * (cap + spill), 3), dtype=np.uint32)
        for q in range(parts):
            sent = np.uint64(range_start(q + 1, parts))
            for t in range(cap + spill):
                slot = q * cap + t if t < cap else parts * cap + q * spill + (t - cap)
                if t < c[q]:
                    kk, vv = k[off[q] + t], (p[off[q] + t] + np.uint64(file0)) & np.uint64(0xFFFFFFFF)
                else:
                    kk, vv = sent, np.uint64(0xFFFFFFFF)
                rows[slot] = [kk & np.uint64(0xFFFFFFFF), kk >> np.uint64(32), vv]
        overflow = torch.tensor([int((c > cap + spill).any())], dtype=torch.int32)
        r = torch.from_numpy(rows.view(np.int32))
        return r[:parts * cap].contiguous(), r[parts * cap:].contiguous(), overflow

    def split_fixed(self, rows, sentinel):
        k, v = self.split(rows)
        ku = k.numpy().view(np.uint64)
        hit = ku == np.uint64(sentinel)
        j = np.arange(len(ku), dtype=np.uint64)
        ku[hit] = np.uint64(sentinel) + j[hit]  # distinct keys, outside the receiver's range
        return k, v, torch.tensor([int(hit.sum())], dtype=torch.int64)

    def unpack_fixed(self, back, spill_back, pos, counts, parts, cap, spill):
        b, sb, p, c = back.numpy().view(np.uint32), spill_back.numpy().view(np.uint32), pos.numpy(), counts.numpy()
        off = np.concatenate([[0], np.cumsum(c)[:-1]])
        rep = np.empty(len(p), dtype=np.int64)
        for q in range(parts):
            for t in range(min(int(c[q]), cap + spill)):
                rep[p[off[q] + t]] = b[q * cap + t] if t < cap else sb[q * spill + t - cap]
        return torch.from_numpy(rep)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, all_keys, per, q, capacity):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from spacedrive_amd.shard import sharded_group
    lo, hi = rank * per, min(len(all_keys), (rank + 1) * per)
    keys = torch.from_numpy(all_keys[lo:hi].view(np.int64).copy())
    res = sharded_group(keys, lo, HostOps(rank), capacity=capacity)
    overflowed = None if res.overflow is None else int(res.overflow.item())
    res.resolve()
    q.put((rank, res.rep.numpy().tolist(), res.objects, overflowed))
    dist.barrier()
    dist.destroy_process_group()


def run_sharded(all_keys: np.ndarray, world: int, capacity=None, want_overflow=None):
    per = (len(all_keys) + world - 1) // world
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, all_keys, per, q, capacity))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    rep = sum((o[1] for o in out), [])
    assert len({o[2] for o in out}) == 1
    if want_overflow is not None:
        assert {o[3] for o in out} == {int(want_overflow)}
    return np.array(rep), out[0][2]


def boundary_keys(rng, world, n_pool, n):
    pool = rng.integers(0, 2 ** 64, n_pool, dtype=np.uint64)
    pool[:5] = [0, 1, 2 ** 63, 2 ** 63 - 1, 2 ** 64 - 1]  # range-boundary keys
    from spacedrive_amd.shard import range_start
    for r in range(1, world):  # every range's first key, its predecessor (= sentinels)
        b = range_start(r, world)
        pool[5 + 2 * r: 7 + 2 * r] = [b, b - 1]
    return pool[rng.integers(0, len(pool), n)]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_group_matches_canonical(world, oracle):
    rng = np.random.default_rng(world)
    keys = boundary_keys(rng, world, 900, 2500)
    rep, objects = run_sharded(keys, world)
    orep, oobj = oracle.group_canonical(keys)
    assert objects == oobj
    assert (rep == orep.astype(np.int64)).all()


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_group_fixed_capacity(world, oracle):
    """The sync-free exchange (fixed per-peer capacity, sentinel rows in unused slots,
    spill blocks): same grouping as the canonical one, keys equal to every sentinel
    (the first key of each range) included, no overflow for uniform keys."""
    from spacedrive_amd.shard import fixed_capacity
    rng = np.random.default_rng(10 + world)
    keys = boundary_keys(rng, world, 1500, 4000)
    per = (len(keys) + world - 1) // world
    rep, objects = run_sharded(keys, world, capacity=fixed_capacity(per, world), want_overflow=0)
    orep, oobj = oracle.group_canonical(keys)
    assert objects == oobj
    assert (rep == orep.astype(np.int64)).all()


def test_sharded_group_fixed_capacity_overflow_falls_back(oracle):
    """A heavily duplicated library (many copies of one file: all on one rank's range)
    overflows the fixed capacity; the max-reduced flag makes every rank redo the step with
    the exact exchange, and the result is still the canonical grouping."""
    rng = np.random.default_rng(33)
    keys = rng.integers(0, 2 ** 64, 3000, dtype=np.uint64)
    keys[::2] = keys[7]  # half the files are one content
    world = 4
    per = (len(keys) + world - 1) // world
    rep, objects = run_sharded(keys, world, capacity=(per // world + 20, 16), want_overflow=1)
    orep, oobj = oracle.group_canonical(keys)
    assert objects == oobj
    assert (rep == orep.astype(np.int64)).all()


def test_range_part_boundaries():
    k = np.array([0, 1, 2 ** 62, 2 ** 63 - 1, 2 ** 63, 3 * 2 ** 62, 2 ** 64 - 1], dtype=np.uint64)
    assert range_part(k, 2).tolist() == [0, 0, 0, 0, 1, 1, 1]
    assert range_part(k, 4).tolist() == [0, 0, 1, 1, 2, 3, 3]
    assert range_part(k, 3).tolist() == [0, 0, 0, 1, 1, 2, 2]
    assert range_part(k, 1).tolist() == [0] * 7
    for parts in (3, 5, 7, 8):
        for x in k.tolist():
            assert range_part(np.array([x], dtype=np.uint64), parts)[0] == (x * parts) >> 64
