#!/usr/bin/env python3
"""Object grouping on one GPU: K4h/K5h (bucket partition + LDS hash min, sd_cas_group_dev)
vs the LSD radix sort + run heads (sd_cas_sort_pairs_dev + sd_cas_group_sorted_dev), at
the bench's per-GPU batch (1.31M keys) and config 4's rank share (12.5M keys), 30 % dups.
Both results are checked against each other; one JSON line per size.
--only hash|lsd: run ONE method only (chain_calls of it, incl. the warm-up call) and no
cross-check — the PMC passes of tools/gpu_r5_pmc_sort.sh attribute every sd_* dispatch of
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
        if only == "hash":
            obj = eng.group(keys, rep)
            t = timed(lambda: eng.group(keys, rep, want_objects=False))
            print(json.dumps({"keys": n, "method": "hash", "objects": obj, "ms": t, "chain_calls": 6}), flush=True)
            continue
        if only == "lsd":
            legacy()
            t = timed(legacy)
            print(json.dumps({"keys": n, "method": "lsd", "ms": t, "chain_calls": 6}), flush=True)
            continue
        obj = eng.group(keys, rep)  # warm + workspace
        t_hash = timed(lambda: eng.group(keys, rep, want_objects=False))
        legacy()
        t_lsd = timed(legacy)
        same = bool(torch.equal(rep, rep2))
        bpk = 36 if n <= 256 * 5632 else (68 if n <= 40_000_000 else 76)  # bench.group_bytes_per_key
        print(json.dumps({"keys": n, "objects": obj, "hash_group_ms": t_hash, "lsd_group_ms": t_lsd,
                          "speedup": t_lsd / t_hash, "hash_gkeys_per_s": n / t_hash / 1e6,
                          "hash_bytes_per_key": bpk,
                          "hash_hbm_gb_per_s_algorithmic": bpk * n / t_hash / 1e6,
                          "identical": same}), flush=True)


if __name__ == "__main__":
    main()
