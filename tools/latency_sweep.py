"""Crossover sweep: lane-per-file kernels (K1/K2) vs chunk-parallel K1L (a wave per file,
and four files per wave) by batch size.

Times sd_cas_hash_sampled_dev / sd_cas_hash_packed_dev with the latency threshold forced
to each path, on torch's current stream (the engine launches there), median of R reps.
Output: one line per (layout, n) with both times and the files/s each reaches.
"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from spacedrive_amd import CasEngine  # noqa: E402

SAMPLED = 57344


def timed(fn, reps=20):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    eng = CasEngine(0)
    q = eng.batch_quantum
    ns = [1, 100, 512, 1024, 2048, 4096, 8192, 16384, 32768, 49152, q, q + 4096, q + q // 2,
          2 * q, 2 * q + 20000, 3 * q, 4 * q, 6 * q]
    if len(sys.argv) > 1:  # explicit batch sizes, in quanta if suffixed with q
        ns = [int(float(x[:-1]) * q) if x.endswith("q") else int(x) for x in sys.argv[1:]]
    nmax = max(ns)
    content = torch.empty(nmax * SAMPLED, dtype=torch.uint8, device="cuda")
    sizes = torch.empty(nmax, dtype=torch.int64, device="cuda")
    eng.synth_sampled(7, 0, nmax, content, sizes, SAMPLED)
    # ragged whole files: synth_small lays out an arena of files <= 100 KiB
    slens = torch.empty(nmax, dtype=torch.int32, device="cuda")
    soffs = torch.empty(nmax, dtype=torch.int64, device="cuda")
    ssizes = torch.empty(nmax, dtype=torch.int64, device="cuda")
    nbytes = eng.synth_small(7, 0, nmax, ssizes, slens, soffs, None)
    arena = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
    eng.synth_small(7, 0, nmax, ssizes, slens, soffs, arena)
    keys = torch.empty(nmax, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    rows = []
    for n in ns:
        row = {"n": n}
        for name, thr, split in (("lane", 0, 0), ("chunkpar", 1 << 40, 1 << 40),
                                 ("chunkpar16", 1 << 40, 0)):
            eng.set_latency_threshold(thr, thr)
            eng.set_chunkpar_split(split, split)
            t = timed(lambda: eng.hash_sampled(content, sizes[:n], keys, stride=SAMPLED, n=n))
            row[f"sampled_{name}_ms"] = round(t, 4)
            t = timed(lambda: eng.hash_packed(arena, soffs[:n], slens[:n], ssizes[:n], keys[:n]))
            row[f"packed_{name}_ms"] = round(t, 4)
        eng.set_latency_threshold()
        eng.set_chunkpar_split()
        row["sampled_auto_ms"] = round(timed(lambda: eng.hash_sampled(content, sizes[:n], keys, stride=SAMPLED, n=n)), 4)
        row["packed_auto_ms"] = round(timed(lambda: eng.hash_packed(arena, soffs[:n], slens[:n], ssizes[:n], keys[:n])), 4)
        rows.append(row)
        print(json.dumps(row), flush=True)
    eng.set_latency_threshold()
    eng.set_chunkpar_split()


if __name__ == "__main__":
    main()
