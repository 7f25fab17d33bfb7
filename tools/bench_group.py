#!/usr/bin/env python3
"""Object grouping on one GPU: K4h/K5h (bucket partition + LDS hash min, sd_cas_group_dev)
vs the LSD radix sort + run heads, at the bench's per-GPU batch (1.31M keys) and config 4's
rank share (12.5M keys), 30 % dups.  The LSD grouping is timed two ways: as the product runs
it (sd_cas_group_dev with SD_CAS_GROUP_SORT: the iota sort lays down rep[i] = i in its first
pass and the runs kernel stores only duplicates) and through the public pair API
(sd_cas_sort_pairs_dev + sd_cas_group_sorted_dev, which stores every rep).  All results are
checked against each other; one JSON line per size.
--only hash|lsd|lsdapi: run ONE method only (chain_calls of it, incl. the warm-up call) and no
cross-check — the PMC passes of tools/gpu_r6_pmc_sort.sh attribute every sd_* dispatch of
the process to that method."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spacedrive_amd import CasEngine  # noqa: E402


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    args = sys.argv[1:]
    only = None
    if "--only" in args:
        i = args.index("--only")
        only = args[i + 1]
        del args[i:i + 2]
    eng = CasEngine(0)
    rng = np.random.default_rng(1)
    for n in [int(x) for x in (args or ["1310720", "12500000"])]:
        uniq = rng.integers(0, 2 ** 64, int(n * 0.7), dtype=np.uint64)
        keys_h = np.concatenate([uniq, uniq[rng.integers(0, len(uniq), n - len(uniq))]])
        rng.shuffle(keys_h)
        keys = torch.from_numpy(keys_h.view(np.int64)).cuda()
        rep = torch.empty(n, dtype=torch.int32, device="cuda")
        rep2 = torch.empty(n, dtype=torch.int32, device="cuda")
        ko = torch.empty_like(keys)
        vo = torch.empty(n, dtype=torch.int32, device="cuda")
        def legacy():
            eng.sort_pairs(keys, None, ko, vo)
            eng.group_sorted(ko, vo, rep2)

        def lsd(out, want=False):
            eng.set_group_method(eng.GROUP_SORT)
            try:
                return eng.group(keys, out, want_objects=want)
            finally:
                eng.set_group_method(eng.GROUP_AUTO)
        if only == "hash":
            obj = eng.group(keys, rep)
            t = timed(lambda: eng.group(keys, rep, want_objects=False))
            print(json.dumps({"keys": n, "method": "hash", "objects": obj, "ms": t, "chain_calls": 6}), flush=True)
            continue
        if only == "lsd":
            obj = lsd(rep, True)
            t = timed(lambda: lsd(rep))
            print(json.dumps({"keys": n, "method": "lsd", "objects": obj, "ms": t, "chain_calls": 6}), flush=True)
            continue
        if only == "lsdapi":
            legacy()
            t = timed(legacy)
            print(json.dumps({"keys": n, "method": "lsdapi", "ms": t, "chain_calls": 6}), flush=True)
            continue
        obj = eng.group(keys, rep)  # warm + workspace
        t_hash = timed(lambda: eng.group(keys, rep, want_objects=False))
        legacy()
        t_api = timed(legacy)
        rep3 = torch.empty(n, dtype=torch.int32, device="cuda")
        obj3 = lsd(rep3, True)
        t_lsd = timed(lambda: lsd(rep3))
        same = bool(torch.equal(rep, rep2)) and bool(torch.equal(rep, rep3)) and obj3 == obj
        bpk = 36 if n <= 256 * 5632 else (68 if n <= 40_000_000 else 76)  # bench.group_bytes_per_key
        print(json.dumps({"keys": n, "objects": obj, "hash_group_ms": t_hash, "lsd_group_ms": t_lsd,
                          "lsd_api_chain_ms": t_api, "speedup": t_lsd / t_hash, "hash_gkeys_per_s": n / t_hash / 1e6,
                          "hash_bytes_per_key": bpk,
                          "hash_hbm_gb_per_s_algorithmic": bpk * n / t_hash / 1e6,
                          "identical": same}), flush=True)


if __name__ == "__main__":
    main()
