"""Profiling driver: synthesize a resident sampled batch and launch K1 a few times.
Used under rocprofv3 (kernel trace / PMC passes); prints kernel-only GB/s."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from spacedrive_amd import CasEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--files", type=int, default=1_250_000)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--group", action="store_true")
ap.add_argument("--fused", action="store_true", help="K1G + bucket tables (hash_group_sampled)")
a = ap.parse_args()
eng = CasEngine(0)
content = torch.empty((a.files, 57344), dtype=torch.uint8, device="cuda")
sizes = torch.empty(a.files, dtype=torch.int64, device="cuda")
keys = torch.empty(a.files, dtype=torch.int64, device="cuda")
rep = torch.empty(a.files, dtype=torch.int32, device="cuda")
ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
eng.synth_sampled(7, 0, a.files, content, sizes, 57344, dup_permille=300)
torch.cuda.synchronize()
for i in range(a.iters):
    t = time.perf_counter()
    if a.fused:
        eng.hash_group_sampled(content, sizes, keys, rep, ovf, want_objects=False)
    else:
        eng.hash_sampled(content, sizes, keys)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"iter {i}: {dt*1e3:.2f} ms  {a.files*57352/dt/1e9:.0f} GB/s  {a.files/dt/1e6:.1f} M files/s", flush=True)
    if a.group:
        eng.group(keys, rep)
# keys digest: variants of the kernel must agree (A/B parity)
k = keys.cpu().numpy().view("uint64")
print(f"keys_digest {int((k * 0x9E3779B97F4A7C15).sum() & 0xFFFFFFFFFFFFFFFF):016x}", flush=True)
