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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, all_keys, per, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from spacedrive_amd.shard import sharded_group
    lo, hi = rank * per, min(len(all_keys), (rank + 1) * per)
    keys = torch.from_numpy(all_keys[lo:hi].view(np.int64).copy())
    res = sharded_group(keys, lo, HostOps())
    q.put((rank, res.rep.numpy().tolist(), res.objects))
    dist.barrier()
    dist.destroy_process_group()


def run_sharded(all_keys: np.ndarray, world: int):
    per = (len(all_keys) + world - 1) // world
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, all_keys, per, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    rep = sum((o[1] for o in out), [])
    assert len({o[2] for o in out}) == 1
    return np.array(rep), out[0][2]


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_group_matches_canonical(world, oracle):
    rng = np.random.default_rng(world)
    pool = rng.integers(0, 2 ** 64, 900, dtype=np.uint64)
    pool[:5] = [0, 1, 2 ** 63, 2 ** 63 - 1, 2 ** 64 - 1]  # range-boundary keys
    keys = pool[rng.integers(0, len(pool), 2500)]
    rep, objects = run_sharded(keys, world)
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
