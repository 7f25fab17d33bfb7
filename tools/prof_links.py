#!/usr/bin/env python3
"""Object-link emission of a whole identifier job (sd_cas_identifier_links_ex_dev) on 1M and
10M device-resident rows (30 % duplicate keys, 0.1 % errored and 0.1 % emptied rows),
chunk 100 — wall time per call (blocking), median of 5, in three forms: a fresh library,
seeded with the library's Objects for 20 % of the keys, and with 1 % of the rows already
owning an Object (the watcher's create-empty-then-write rows: the stable key sort + two
segmented-min scans of links.hip); the last also checked against the closed form on 1M."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from spacedrive_amd import CasEngine  # noqa: E402

eng = CasEngine(0)
rng = np.random.default_rng(4)
for n in (1_000_000, 10_000_000):
    pool = rng.integers(0, 2 ** 64, int(n * 0.7), dtype=np.uint64)
    keys = pool[rng.integers(0, len(pool), n)]
    state = np.zeros(n, dtype=np.uint8)
    state[rng.random(n) < 0.001] = 1
    state[rng.random(n) < 0.001] = 2
    dk = torch.from_numpy(keys.view(np.int64)).cuda()
    ds = torch.from_numpy(state).cuda()
    sk = pool[rng.random(len(pool)) < 0.2]
    so = rng.integers(0, 2 ** 31 - 1, len(sk)).astype(np.uint32)
    seeds = (torch.from_numpy(sk.view(np.int64)).cuda(), torch.from_numpy(so.view(np.int32)).cuda())
    pre = np.full(n, 0xFFFFFFFF, np.uint32)
    own = rng.random(n) < 0.01
    pre[own] = rng.integers(0, 2 ** 31 - 1, int(own.sum())).astype(np.uint32)
    dpre = torch.from_numpy(pre.view(np.int32)).cuda()
    for form, kw in (("fresh", {}), ("seeded", {"existing": seeds}),
                     ("seeded+pre_objects", {"existing": seeds, "pre_objects": dpre})):
        eng.identifier_links(dk, ds, **kw)
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            _, _, _, counts = eng.identifier_links(dk, ds, **kw)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        print(json.dumps({"rows": n, "form": form, "steps": int(len(counts)),
                          "ms": float(np.median(ts) * 1e3),
                          "rows_per_s": n / float(np.median(ts))}), flush=True)
