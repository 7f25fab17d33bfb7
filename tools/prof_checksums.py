#!/usr/bin/env python3
"""The validator job over many files (sd_cas_checksums_dev / sd_cas_file_checksums).

Device batches (resident, synthetic): one launch chain per batch, HIP events on the
engine's stream; every digest of a sample checked against the oracle.  Library shapes:
  photos  4,096 buffers of U(1, 8) MiB      (~18 GB)
  docs    262,144 buffers of U(1, 128) KiB  (~17 GB)
  small   1,048,576 buffers of U(0, 16) KiB (~8.6 GB)
  one     one 16 GiB buffer (the K3 single-buffer chain's shape, for comparison)
  small16k .. small256k  16,384 .. 262,144 buffers of U(0, 16) KiB (batch-size sweep)
  docs64  262,144 buffers of U(1, 64) KiB
  skew64k / skew1m  mostly U(0, 4) KiB with 8 % U(96, 128) KiB / 3 % U(64, 128) KiB
Paths (--paths N): N files of U(0.25, 4) MiB (--path-kib LO HI) on /dev/shm through sd_cas_file_checksums vs
the oracle's file_checksum on 1 thread (hash.rs is single-threaded) and file-parallel on
the host cores.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"photos": (4096, 1 << 20, 8 << 20), "docs": (262144, 1 << 10, 128 << 10),
          "small": (1 << 20, 0, 16 << 10), "one": (1, 16 << 30, 16 << 30),
          # batch-size sweep of the small shape (the lane-per-buffer path's crossover)
          "small16k": (16384, 0, 16 << 10), "small32k": (32768, 0, 16 << 10),
          "small64k": (65536, 0, 16 << 10), "small128k": (131072, 0, 16 << 10),
          "small256k": (262144, 0, 16 << 10), "docs64": (262144, 1 << 10, 64 << 10),
          # skewed libraries: mostly tiny files and a few long ones (n, [(fraction, lo, hi)])
          "skew64k": (65536, [(0.92, 0, 4 << 10), (0.08, 96 << 10, 128 << 10)]),
          "skew1m": (1 << 20, [(0.97, 0, 4 << 10), (0.03, 64 << 10, 128 << 10)])}


def device_batch(eng, orc, name, iters):
    import numpy as np
    import torch
    spec = SHAPES[name]
    n = spec[0]
    rng = np.random.default_rng(5)
    if isinstance(spec[1], list):  # a mixture, shuffled
        parts = [rng.integers(lo, hi + 1, int(round(fr * n)), dtype=np.uint64) for fr, lo, hi in spec[1]]
        lens = np.concatenate(parts)[:n]
        lens = np.concatenate([lens, np.zeros(n - len(lens), dtype=np.uint64)])[rng.permutation(n)]
    else:
        lo, hi = spec[1], spec[2]
        lens = rng.integers(lo, hi + 1, n, dtype=np.uint64) if hi > lo else np.full(n, lo, dtype=np.uint64)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum((lens[:-1] + 127) // 128 * 128)
    total = int(offs[-1] + lens[-1])
    ab = (total + 127) // 128 * 128 + 128
    arena = torch.empty(ab, dtype=torch.uint8, device="cuda")
    eng.synth_stream(77, 0, 0, ab // 8 * 8, arena)
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_lens = torch.from_numpy(lens.view(np.int64)).cuda()
    out = torch.zeros((n, 32), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    eng.checksums_dev(arena, d_offs, d_lens, out, stream=s.cuda_stream)
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        eng.checksums_dev(arena, d_offs, d_lens, out, stream=s.cuda_stream)
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ms = float(np.median(ts))
    got = out.cpu().numpy()
    idx = sorted(set(rng.integers(0, n, min(n, 64)).tolist()) | {0, n - 1})
    ok = True
    for i in idx:
        o, L = int(offs[i]), int(lens[i])
        if L > (1 << 30):  # the single 16 GiB buffer: the oracle's tree-parallel hash
            want = orc.blake3_mt(arena[o:o + L].cpu().numpy(), 16)
        else:
            want = orc.blake3(arena[o:o + L].cpu().numpy().tobytes())
        ok &= got[i].tobytes() == want
    comps = int((lens // 64).sum() + (lens // 1024).sum())
    k3 = None
    if n == 1:  # the single-buffer K3 chain on the same bytes, for comparison
        L = int(lens[0])
        t3 = []
        for _ in range(iters):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            d3 = eng.checksum_dev(arena, L, stream=s.cuda_stream)
            b.record(s)
            b.synchronize()
            t3.append(a.elapsed_time(b))
        k3 = {"ms": float(np.median(t3)), "gb_per_s": L / (float(np.median(t3)) / 1e3) / 1e9,
              "same_digest": d3 == got[0].tobytes().hex()}
    del arena, out
    torch.cuda.empty_cache()
    return {"shape": name, "buffers": n, "bytes": int(lens.sum()), "ms": ms,
            "ms_all": ts, "gb_per_s": float(lens.sum()) / (ms / 1e3) / 1e9,
            "buffers_per_s": n / (ms / 1e3),
            "valu_slot_frac": comps * 1014 / 64 / (ms / 1e3) / (1024 * 2.4e9 / 2),
            "parity_sample": len(idx), "parity": bool(ok), "k3_same_bytes": k3}


def paths_run(eng, orc, n, root, nruns=3, lo_kb=256, hi_kb=4096):
    import numpy as np
    rng = np.random.default_rng(6)
    os.makedirs(root, exist_ok=True)
    sizes = rng.integers(lo_kb << 10, hi_kb << 10, n)
    paths = []
    for i, L in enumerate(sizes):
        p = os.path.join(root, f"v{i}")
        with open(p, "wb") as fh:
            fh.write(orc.fill_content_range(88, i, 0, int(L) // 8 * 8).tobytes())
        paths.append(p)
    total = int(sum(int(L) // 8 * 8 for L in sizes))
    eng.file_checksums(paths[:8])
    runs = []  # runs[0]: the first pass over the just-written files (cold page-cache access)
    for _ in range(nruns):
        t = time.perf_counter()
        got, errs = eng.file_checksums(paths)
        runs.append(time.perf_counter() - t)
    gpu_s = min(runs)
    warm = sorted(runs[1:]) or runs
    # CPU: hash.rs is one thread per file; the job is one file per step
    m1 = min(n, 64)
    t = time.perf_counter()
    one = [orc.file_checksum(p) for p in paths[:m1]]
    cpu1_s = (time.perf_counter() - t) * n / m1
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    t = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        allc = list(ex.map(orc.file_checksum, paths))
    cpun_s = time.perf_counter() - t
    parity = got == allc and got[:m1] == one and not any(errs)
    # the same hash.rs loop with the BLAKE3 team's C library (SIMD, what the crate does)
    official = None
    try:
        from oracle.pyoracle import ExtBlake3
        ext = ExtBlake3()
        t = time.perf_counter()
        o1, _ = ext.file_checksums(paths[:m1], 1)
        e1 = (time.perf_counter() - t) * n / m1
        t = time.perf_counter()
        on, _ = ext.file_checksums(paths, threads)
        en = time.perf_counter() - t
        official = {"library": f"BLAKE3 C {ext.version()} (libclang-cpp.so)",
                    "cpu_1thread_gb_per_s": total / e1 / 1e9,
                    "cpu_all_gb_per_s": total / en / 1e9, "parity": on == got and o1 == got[:m1]}
    except OSError:
        pass
    for p in paths:
        os.unlink(p)
    return {"files": n, "size_kib": [lo_kb, hi_kb], "bytes": total, "gpu_s": gpu_s, "gpu_s_runs": runs, "gpu_gb_per_s": total / gpu_s / 1e9,
            "gpu_files_per_s": n / gpu_s,
            "cold_first_pass_gb_per_s": total / runs[0] / 1e9,
            "warm_median_gb_per_s": total / warm[len(warm) // 2] / 1e9, "cpu_1thread_gb_per_s": total / cpu1_s / 1e9,
            "cpu_threads": threads, "cpu_all_gb_per_s": total / cpun_s / 1e9,
            "cpu_note": "cpu_* = the oracle's portable C (scalar); official_c = the C library",
            "official_c": official, "parity": bool(parity)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append", default=None)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--paths", type=int, default=0)
    ap.add_argument("--path-runs", type=int, default=3)
    ap.add_argument("--path-kib", type=int, nargs=2, default=[256, 4096], metavar=("LO", "HI"),
                    help="file sizes U(LO, HI) KiB (default: the 2,000-file set's U(0.25, 4) MiB)")
    ap.add_argument("--no-device", action="store_true", help="paths only")
    ap.add_argument("--root", default="/dev/shm/sdcas_validator")
    a = ap.parse_args()
    from spacedrive_amd import CasEngine
    from oracle.pyoracle import Oracle
    eng, orc = CasEngine(0), Oracle()
    for name in [] if a.no_device else a.shape or ["photos", "docs", "small", "one"]:
        print(json.dumps(device_batch(eng, orc, name, a.iters)), flush=True)
    if a.paths:
        print(json.dumps(paths_run(eng, orc, a.paths, a.root, a.path_runs, a.path_kib[0], a.path_kib[1])), flush=True)


if __name__ == "__main__":
    main()
