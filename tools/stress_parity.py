#!/usr/bin/env python3
"""Randomised parity stress for the LDS-heavy kernels (a rare cross-wave race showed up
only once in 10^7 keys): for --seconds, draw random sizes and key patterns and
check, every iteration,
  * sd_cas_group_dev (hash grouping; every 4th iteration the forced LSD path) against the
    canonical rep from numpy's stable sort (rep[i] = smallest index with the same key),
  * sd_cas_group_min_dev with random u32 values against numpy,
  * sd_cas_sort_pairs_dev against numpy's stable argsort,
  * (--validator) sd_cas_checksums_dev over a random batch of ragged buffers of every size
    class against the oracle's BLAKE3; every 8th iteration a batch of 65,536-80,000 buffers
    (the lane-per-buffer path, mostly <= 128 KiB).
Key patterns: uniform 64-bit, few distinct keys (hot keys), small integers (not uniform
after any mix), bucket-sorted runs.  Prints one JSON line per iteration and a summary.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def canonical(keys, vals=None):
    import numpy as np
    n = len(keys)
    v = np.arange(n, dtype=np.uint64) if vals is None else vals.astype(np.uint64)
    # sort by (key, val): the run head holds the minimum value
    order = np.lexsort((v, keys))
    sk = keys[order]
    head = np.ones(n, dtype=bool)
    head[1:] = sk[1:] != sk[:-1]
    run = np.cumsum(head) - 1
    first_val = v[order][head]
    out = np.empty(n, dtype=np.uint64)
    out[order] = first_val[run]
    return out, int(head.sum())


def draw_keys(rng, n, pattern):
    import numpy as np
    if pattern == "uniform":
        k = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
        d = rng.integers(0, n, n // 3)
        k[d] = k[rng.integers(0, n, len(d))]
        return k
    if pattern == "hot":
        distinct = rng.integers(0, 2 ** 64, max(1, int(rng.integers(1, 64))), dtype=np.uint64)
        k = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
        m = rng.random(n) < rng.uniform(0.05, 0.6)
        k[m] = distinct[rng.integers(0, len(distinct), int(m.sum()))]
        return k
    if pattern == "small":
        return rng.integers(0, max(2, n // int(rng.integers(1, 8))), n).astype(np.uint64)
    # "sorted": bucket-sorted runs of a uniform draw
    k = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
    return np.sort(k)[rng.permutation(n) if rng.random() < 0.3 else slice(None)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180)
    ap.add_argument("--max-n", type=int, default=4_000_000)
    ap.add_argument("--seed", type=int, default=2026)
    ap.add_argument("--validator", action="store_true",
                    help="also stress sd_cas_checksums_dev: random batches of ragged buffers vs the oracle")
    a = ap.parse_args()
    import numpy as np
    import torch
    from spacedrive_amd import CasEngine
    from oracle.pyoracle import Oracle
    eng = CasEngine(0)
    orc = Oracle() if a.validator else None
    rng = np.random.default_rng(a.seed)
    t_end = time.time() + a.seconds
    it = fails = 0
    while time.time() < t_end:
        n = int(rng.integers(1, a.max_n + 1)) if rng.random() < 0.8 else int(rng.integers(1, 5000))
        pattern = ["uniform", "hot", "small", "sorted"][it % 4]
        keys = draw_keys(rng, n, pattern)
        dk = torch.from_numpy(keys.view(np.int64)).cuda()
        res = {"it": it, "n": n, "pattern": pattern}
        # grouping (hash; every 4th iteration the LSD path)
        method = 2 if it % 4 == 3 else 0
        eng.set_group_method(method)
        rep = torch.empty(n, dtype=torch.int32, device="cuda")
        objects = eng.group(dk, rep)
        want, wobj = canonical(keys)
        res["group"] = bool(objects == wobj and (rep.cpu().numpy().astype(np.uint64) == want).all())
        eng.set_group_method(0)
        # group_min with random values
        vals = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        obj2 = eng.group_min(dk, torch.from_numpy(vals.view(np.int32)).cuda(), out)
        want2, wobj2 = canonical(keys, vals)
        res["group_min"] = bool(obj2 == wobj2 and (out.cpu().numpy().view(np.uint32).astype(np.uint64) == want2).all())
        # stable sort
        ko = torch.empty(n, dtype=torch.int64, device="cuda")
        vo = torch.empty(n, dtype=torch.int32, device="cuda")
        eng.sort_pairs(dk, None, ko, vo)
        order = np.argsort(keys, kind="stable")
        res["sort"] = bool((vo.cpu().numpy() == order).all())
        if orc is not None:
            # a batch of ragged buffers across every size class (<=16, 17-64, 65-256 and
            # > 256 chunks), shuffled arena order
            big = it % 8 == 7
            nb = int(rng.integers(65536, 80000)) if big else int(rng.integers(1, 400))
            cls = rng.choice(4, nb, p=[0.45, 0.3, 0.249, 0.001]) if big else rng.integers(0, 4, nb)
            hi = np.array([16 << 10, 64 << 10, 128 << 10 if big else 256 << 10, 3 << 20])[cls]
            lens = (rng.random(nb) * hi).astype(np.uint64)
            offs = np.zeros(nb, dtype=np.uint64)
            o = 0
            for i in rng.permutation(nb):
                offs[i] = o
                o += (int(lens[i]) + 15) // 16 * 16 + (0 if big else 16 * int(rng.integers(0, 3)))
            ab = (o + 16) // 8 * 8 + 8
            arena = torch.empty(ab, dtype=torch.uint8, device="cuda")
            eng.synth_stream(a.seed, it, 0, ab, arena)
            host = arena.cpu().numpy()
            out = torch.zeros((nb, 32), dtype=torch.uint8, device="cuda")
            eng.checksums_dev(arena, torch.from_numpy(offs.view(np.int64)).cuda(),
                              torch.from_numpy(lens.view(np.int64)).cuda(), out)
            got = out.cpu().numpy()
            res["checksums"] = all(got[i].tobytes() == orc.blake3(host[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes())
                                   for i in range(nb))
            res["buffers"] = nb
        ok = res["group"] and res["group_min"] and res["sort"] and res.get("checksums", True)
        fails += 0 if ok else 1
        res["ok"] = ok
        print(json.dumps(res), flush=True)
        it += 1
    print(json.dumps({"iterations": it, "failures": fails, "seconds": a.seconds}), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
