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
    (the lane-per-buffer path, mostly <= 128 KiB),
  * (--fused) the fused hash + group chain (K1G + the region tables, blocking form and the
    split form over both region sets) on a random batch of synthetic sampled files with
    random duplication and hot files copied up to 30,000 times: keys against K1, rep against
    the canonical grouping of those keys.
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
    ap.add_argument("--lsd-every", type=int, default=4, help="forced LSD grouping every k-th iteration")
    ap.add_argument("--validator", action="store_true",
                    help="also stress sd_cas_checksums_dev: random batches of ragged buffers vs the oracle")
    ap.add_argument("--fused", action="store_true",
                    help="also stress the fused K1G + region-table chain (sd_cas_hash_group_sampled_dev)")
    ap.add_argument("--fused-max", type=int, default=1_310_720)
    a = ap.parse_args()
    import numpy as np
    import torch
    from spacedrive_amd import CasEngine
    from oracle.pyoracle import Oracle
    eng = CasEngine(0)
    orc = Oracle() if a.validator else None
    rng = np.random.default_rng(a.seed)
    if a.fused:
        F = a.fused_max
        fcontent = torch.empty((F, 57344), dtype=torch.uint8, device="cuda")
        fsizes = torch.empty(F, dtype=torch.int64, device="cuda")
        fkeys = torch.empty(F, dtype=torch.int64, device="cuda")
        fkeys1 = torch.empty(F, dtype=torch.int64, device="cuda")
        freps = [torch.empty(F, dtype=torch.int32, device="cuda") for _ in range(2)]
        fovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    t_end = time.time() + a.seconds
    it = fails = 0
    while time.time() < t_end:
        n = int(rng.integers(1, a.max_n + 1)) if rng.random() < 0.8 else int(rng.integers(1, 5000))
        pattern = ["uniform", "hot", "small", "sorted"][it % 4]
        keys = draw_keys(rng, n, pattern)
        dk = torch.from_numpy(keys.view(np.int64)).cuda()
        res = {"it": it, "n": n, "pattern": pattern}
        # grouping (hash; every 4th iteration the LSD path)
        # the forced LSD path every 4th iteration (--lsd-every 1: every iteration; a pattern
        # per iteration still cycles through all four)
        method = 2 if it % a.lsd_every == a.lsd_every - 1 else 0
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
        if a.fused:
            q = eng.batch_quantum  # the fused chain takes whole quanta (else: the two calls)
            fused_shape = it % 2 == 1 or rng.random() < 0.7
            fn = (q * int(rng.integers(1, F // q + 1)) if fused_shape
                  else int(rng.integers(1, F + 1)))
            c, sz = fcontent[:fn], fsizes[:fn]
            eng.synth_sampled(a.seed + it, 0, fn, c, sz, 57344, dup_permille=int(rng.integers(0, 900)))
            hot = []
            if it % 3 == 0 and fn > 64:  # hot files: one file copied many times
                for h in range(int(rng.integers(1, 4))):
                    copies = int(rng.integers(2, min(30_000, fn // 2) + 1))
                    src = int(rng.integers(0, fn))
                    idx = torch.from_numpy(rng.choice(fn, copies, replace=False)).cuda()
                    c[idx] = c[src].clone()
                    sz[idx] = sz[src].clone()
                    hot.append(copies)
            torch.cuda.synchronize()
            eng.hash_sampled(c, sz, fkeys1[:fn])
            fovf.zero_()
            torch.cuda.synchronize()
            if it % 2 == 0 or fn % q:  # blocking form
                fobj = eng.hash_group_sampled(c, sz, fkeys[:fn], freps[0][:fn], fovf)
                frep = freps[0][:fn]
            else:  # split form, two batches in flight over the two region sets
                eng.hash_regions_sampled(c, sz, fkeys[:fn], freps[0][:fn], fovf)
                eng.group_regions(fn, freps[0][:fn], want_objects=False)
                eng.hash_regions_sampled(c, sz, fkeys[:fn], freps[1][:fn], fovf)
                fobj = eng.group_regions(fn, freps[1][:fn])
                frep = freps[1][:fn]
                res["split_sets_equal"] = bool(torch.equal(freps[0][:fn], freps[1][:fn]))
            torch.cuda.synchronize()
            kk = fkeys[:fn].cpu().numpy().view(np.uint64)
            fwant, fwobj = canonical(kk)
            res["fused"] = bool((fkeys[:fn] == fkeys1[:fn]).all().item() and fobj == fwobj and
                                (frep.cpu().numpy().astype(np.uint64) == fwant).all() and
                                res.get("split_sets_equal", True))
            res.update({"fused_n": fn, "fused_hot": hot, "fused_overflow": int(fovf.item())})
        ok = (res["group"] and res["group_min"] and res["sort"] and res.get("checksums", True)
              and res.get("fused", True))
        fails += 0 if ok else 1
        res["ok"] = ok
        print(json.dumps(res), flush=True)
        it += 1
    print(json.dumps({"iterations": it, "failures": fails, "seconds": a.seconds}), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
