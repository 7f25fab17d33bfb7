#!/usr/bin/env python3
"""K2 alone on BASELINE config 2's shape (1M whole-file messages, sizes uniform 1..102,400,
resident in HBM) for the rocprofv3 PMC passes of tools/pmc_valu.sh: the length sort + K2
launches only, HIP events on the default stream.  Prints the median ms."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spacedrive_amd import CasEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--files", type=int, default=1_000_000)
ap.add_argument("--iters", type=int, default=3)
a = ap.parse_args()
eng = CasEngine(0)
n = a.files
sizes = torch.empty(n, dtype=torch.int64, device="cuda")
lens = torch.empty(n, dtype=torch.int32, device="cuda")
offs = torch.empty(n, dtype=torch.int64, device="cuda")
nbytes = eng.synth_small(11, 0, n, sizes, lens, offs, None)
arena = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
eng.synth_small(11, 0, n, sizes, lens, offs, arena)
keys = torch.empty(n, dtype=torch.int64, device="cuda")
ts = []
for _ in range(a.iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    eng.hash_packed(arena, offs, lens, sizes, keys)
    e.record()
    e.synchronize()
    ts.append(s.elapsed_time(e))
kh = keys.cpu().numpy().view(np.uint64)
digest = int(np.bitwise_xor.reduce(kh * np.uint64(0x9E3779B97F4A7C15) + np.arange(n, dtype=np.uint64)))
print(f"k2 {n} files: median {float(np.median(ts)):.3f} ms  all {[round(t, 3) for t in ts]}  "
      f"keys digest {digest:016x}", flush=True)
