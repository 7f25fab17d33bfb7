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


class HostOps:
    """Test double of HipShardOps: numpy stable sort + run heads, same contracts."""

    def sort_pairs(self, keys, vals):
        k = keys.numpy().view(np.uint64)
        order = np.argsort(k, kind="stable")
        v = order if vals is None else vals.numpy()[order]
        return (torch.from_numpy(k[order].view(np.int64).copy()),
                torch.from_numpy(v.astype(np.int32)))

    def group_sorted(self, skeys, svals):
        k = skeys.numpy()
        v = svals.numpy()
        rep = np.empty(len(k), dtype=np.int32)
        head = 0
        objects = 0
        for i in range(len(k)):
            if i == 0 or k[i] != k[i - 1]:
                head = i
                objects += 1
            rep[v[i]] = v[head]
        return torch.from_numpy(rep), objects


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


def test_key_range_splits_boundaries():
    from spacedrive_amd.shard import key_range_splits
    k = np.array([0, 1, 2 ** 62, 2 ** 63 - 1, 2 ** 63, 3 * 2 ** 62, 2 ** 64 - 1], dtype=np.uint64)
    t = torch.from_numpy(np.sort(k).view(np.int64).copy())
    assert key_range_splits(t, 2).tolist() == [4, 3]
    assert key_range_splits(t, 4).tolist() == [2, 2, 1, 2]
    assert key_range_splits(t, 3).tolist() == [3, 2, 2]
    assert key_range_splits(t, 1).tolist() == [7]
