"""K2 diagnosis: the packed kernel on (a) K1's uniform sampled layout, (b) 1M ragged
whole-file messages (config 2).  Prints per-variant kernel ms (HIP events) so the K2/K1
gap can be attributed to code structure vs ragged lengths."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spacedrive_amd import CasEngine  # noqa: E402


def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


eng = CasEngine(0)
n = 500_000
content = torch.empty((n, 57344), dtype=torch.uint8, device="cuda")
sizes = torch.empty(n, dtype=torch.int64, device="cuda")
keys = torch.empty(n, dtype=torch.int64, device="cuda")
keys2 = torch.empty(n, dtype=torch.int64, device="cuda")
eng.synth_sampled(3, 0, n, content, sizes, 57344)
offs = torch.arange(n, dtype=torch.int64, device="cuda") * 57344
lens = torch.full((n,), 57344, dtype=torch.int32, device="cuda")
eng.hash_sampled(content, sizes, keys)
eng.hash_packed(content, offs, lens, sizes, keys2)
torch.cuda.synchronize()
assert torch.equal(keys, keys2)
print(f"uniform 57344 x {n}: K1 {timed(lambda: eng.hash_sampled(content, sizes, keys)):.2f} ms   "
      f"K2 {timed(lambda: eng.hash_packed(content, offs, lens, sizes, keys2)):.2f} ms", flush=True)
del content
torch.cuda.empty_cache()

m = 1_000_000
sz = torch.empty(m, dtype=torch.int64, device="cuda")
ln = torch.empty(m, dtype=torch.int32, device="cuda")
of = torch.empty(m, dtype=torch.int64, device="cuda")
nb = eng.synth_small(11, 0, m, sz, ln, of, None)
arena = torch.empty(nb + 64, dtype=torch.uint8, device="cuda")
eng.synth_small(11, 0, m, sz, ln, of, arena)
k = torch.empty(m, dtype=torch.int64, device="cuda")
print(f"ragged 1M: K2 (windowed length sort) {timed(lambda: eng.hash_packed(arena, of, ln, sz, k)):.2f} ms",
      flush=True)

# (c) packing-alignment A/B: the same 1M files with every content at a 16-B aligned offset
# (the packing before this round's change) — a K2 line pair then straddles two 128-B
# cache lines; synth_small itself packs at 128 B
ref = k.clone()
al = ((ln.to(torch.int64) + 15) // 16) * 16
of16 = torch.cumsum(al, 0) - al
nb16 = int(al.sum().item()) + 128
del arena
torch.cuda.empty_cache()
arena16 = torch.empty(nb16, dtype=torch.uint8, device="cuda")
eng.synth_small_content(11, 0, m, of16, ln, arena16)
eng.hash_packed(arena16, of16, ln, sz, k)
torch.cuda.synchronize()
assert torch.equal(k, ref), "16-B packed layout changed the cas keys"
print(f"ragged 1M, 16-B packed offsets: K2 {timed(lambda: eng.hash_packed(arena16, of16, ln, sz, k)):.2f} ms",
      flush=True)
