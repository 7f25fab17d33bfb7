#!/usr/bin/env python3
"""Measures the BASELINE.json configs other than bench.py's headline (one JSON line each).

  --config 1  10k files (log-uniform 1 KiB..10 MiB) on tmpfs: GPU drop-in
              (pread gather at the cas.rs offsets -> pinned -> K1/K2) vs the CPU oracle
              (gather + hash), 1 thread and all cores.
  --config 2  1M whole-file messages (size uniform 1..102,400) resident in HBM: K2
              (length sort + hash), plus the CPU oracle on a sample.
  --config 3e end-to-end sampled path from pinned host memory (PCIe-inclusive), K1 with
              H2D of batch k+1 overlapping hashing of batch k.
  --config 4  one rank's share of the 100M-file library (12.5M files, 30 % duplicates):
              K1 over resident batches, then Object grouping of all 12.5M keys.
  --config 4full  the whole 100M-file library on one GPU: K1 over 80 resident batches,
              grouping of all 100M keys, and the 8-shard key-range exchange path.
  --config 5  validator: full BLAKE3 of a resident buffer (default 64 GiB) with K3, and a
              streamed file_checksum of a file on tmpfs (read + H2D + K3).
Every GPU result is checked against the oracle on (a sample of) the same input.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

THREADS = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
DROPIN_PASSES = int(os.environ.get("SD_CONFIG1_PASSES", "1"))


def emit(d):
    print(json.dumps(d), flush=True)


def config1(eng, orc, n_files: int, root: str):
    rng = np.random.default_rng(1)
    sizes = np.exp(rng.uniform(math.log(1024), math.log(10 * 1024 * 1024), n_files)).astype(np.int64)
    os.makedirs(root, exist_ok=True)
    paths = []
    for i, s in enumerate(sizes):
        p = os.path.join(root, f"f{i:05d}")
        with open(p, "wb") as fh:
            fh.write(rng.integers(0, 256, int(s), dtype=np.uint8).tobytes())
        paths.append(p)
    total = int(sizes.sum())
    try:
        eng.generate_cas_keys_from_paths(paths[:64], sizes[:64])  # warm
        t = time.perf_counter()
        keys, errs = eng.generate_cas_keys_from_paths(paths, sizes)
        gpu_cold = time.perf_counter() - t  # includes growing the pinned staging once
        assert not errs.any()
        # round 6: several timed passes of the drop-in call, median reported
        # (one pass per run gave 629 k-854 k files/s across runs)
        passes = []
        for _ in range(max(1, DROPIN_PASSES)):
            t = time.perf_counter()
            keys2, _ = eng.generate_cas_keys_from_paths(paths, sizes)
            passes.append(time.perf_counter() - t)
            assert (keys2 == keys).all()
        gpu = float(np.median(passes))
        t = time.perf_counter()
        want = [orc.generate_cas_id(p, int(s)) for p, s in zip(paths, sizes)]
        cpu1 = time.perf_counter() - t
        # all cores: the oracle's C gather + AVX-512 hash (16 sampled files per lane group)
        # with files interleaved over THREADS pthreads
        t = time.perf_counter()
        k_mt, st_mt = orc.generate_cas_keys_paths(paths, sizes, THREADS, simd=True)
        cpu_mt = time.perf_counter() - t
        ok = all(f"{k:016x}" == w for k, w in zip(keys, want)) and bool((k_mt == keys).all())
        # the reference's own batch shape: identifier_job_step over CHUNK_SIZE = 100 paths
        # (file_identifier/mod.rs:34), one blocking call per chunk; K1L (default threshold)
        # vs forcing the lane-per-file kernels
        step, step_med = {}, {}
        for name, thr in (("k1l", None), ("lane", 0)):
            eng.set_latency_threshold(thr, thr)
            ts = []
            for i in range(0, n_files, 100):
                t = time.perf_counter()
                k, e = eng.generate_cas_keys_from_paths(paths[i:i + 100], sizes[i:i + 100])
                ts.append(time.perf_counter() - t)
                ok = ok and bool((k == keys[i:i + 100]).all())
            step[name] = float(np.mean(ts)) * 1e3
            step_med[name] = float(np.median(ts)) * 1e3
        eng.set_latency_threshold()
        # the CPU oracle at the same step shape: 100 paths per call, gather + AVX-512 hash on
        # THREADS pthreads (created per call), and on one thread (the reference's job hashes
        # its step on one task, mod.rs:105-147)
        cpu_step = {}
        for name, thr in (("all_cores", THREADS), ("1thread", 1)):
            ts = []
            for i in range(0, n_files, 100):
                t = time.perf_counter()
                k, _ = orc.generate_cas_keys_paths(paths[i:i + 100], sizes[i:i + 100], thr, simd=True)
                ts.append(time.perf_counter() - t)
                ok = ok and bool((k == keys[i:i + 100]).all())
            cpu_step[name] = {"mean": float(np.mean(ts)) * 1e3, "median": float(np.median(ts)) * 1e3}
        # the BLAKE3 team's C library after cas.rs's reads (what the crate's SIMD does per
        # file): one thread, all cores, and the 100-path step on all cores
        official = None
        try:
            from oracle.pyoracle import ExtBlake3
            ext = ExtBlake3()
            t = time.perf_counter()
            ko1, _ = ext.cas_keys_paths(paths, sizes, 1)
            o1 = time.perf_counter() - t
            t = time.perf_counter()
            kon, _ = ext.cas_keys_paths(paths, sizes, THREADS)
            on = time.perf_counter() - t
            ts = []
            for i in range(0, n_files, 100):
                t = time.perf_counter()
                ext.cas_keys_paths(paths[i:i + 100], sizes[i:i + 100], THREADS)
                ts.append(time.perf_counter() - t)
            official = {"library": f"BLAKE3 C {ext.version()} (libclang-cpp.so)",
                        "files_per_s_1thread": n_files / o1, "files_per_s_all_cores": n_files / on,
                        "step_100_ms_all_cores_median": round(float(np.median(ts)) * 1e3, 3),
                        "parity": bool((ko1 == keys).all() and (kon == keys).all())}
        except OSError:
            pass
        emit({"config": 1, "files": n_files, "bytes_on_disk": total, "cpu_official_c": official,
              "small_fraction": float((sizes <= 102400).mean()),
              "gpu_dropin_files_per_s": n_files / gpu, "gpu_s": gpu, "gpu_s_first_call": gpu_cold,
              "gpu_dropin_passes_files_per_s": [round(n_files / x) for x in passes],
              "job_step_100_ms": {k: round(v, 3) for k, v in step.items()},
              "job_step_100_ms_median": {k: round(v, 3) for k, v in step_med.items()},
              "cpu_step_100_ms": {k: {a: round(b, 3) for a, b in v.items()} for k, v in cpu_step.items()},
              "cpu_oracle_1thread_files_per_s": n_files / cpu1,
              "cpu_oracle_all_cores_simd_files_per_s": n_files / cpu_mt, "cpu_threads": THREADS,
              "parity": ok,
              "note": "tmpfs page cache; GPU path = pread gather (16 threads) + pinned H2D + K1/K2"})
    finally:
        shutil.rmtree(root, ignore_errors=True)


def config2(eng, orc, n: int, reps: int):
    import torch
    sizes = torch.empty(n, dtype=torch.int64, device="cuda")
    lens = torch.empty(n, dtype=torch.int32, device="cuda")
    offs = torch.empty(n, dtype=torch.int64, device="cuda")
    nbytes = eng.synth_small(11, 0, n, sizes, lens, offs, None)
    arena = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
    eng.synth_small(11, 0, n, sizes, lens, offs, arena)
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.hash_packed(arena, offs, lens, sizes, keys)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        eng.hash_packed(arena, offs, lens, sizes, keys)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 1e3)
    t = float(np.median(ts))
    msg_bytes = int(lens.sum().item()) + 8 * n
    blocks = ((lens.to(torch.int64) + 8 + 63) // 64)
    chunks = ((lens.to(torch.int64) + 8 + 1023) // 1024)
    comps = int((blocks + chunks - 1).sum().item())
    # oracle on a sample
    idx = np.random.default_rng(2).choice(n, 2000, replace=False)
    h_off = offs.cpu().numpy()
    h_len = lens.cpu().numpy()
    h_sz = sizes.cpu().numpy().view(np.uint64)
    k = keys.cpu().numpy().view(np.uint64)
    sub = [(arena[h_off[i]:h_off[i] + h_len[i]].cpu().numpy().tobytes(), int(h_sz[i])) for i in idx]
    ok = all(orc.cas_key(b, s) == k[i] for (b, s), i in zip(sub, idx))
    t0 = time.perf_counter()
    for b, s in sub:
        orc.cas_key(b, s)
    cpu1 = (time.perf_counter() - t0) / len(sub)
    # SIMD baseline (oracle/cas_fast.c: chunk-parallel AVX-512 per file, the crate's
    # hash_many shape) on all host cores over the first m files of the same arena
    m = min(n, 40000)
    end = int(h_off[m - 1] + h_len[m - 1])
    host = arena[:end + 64].cpu().numpy()
    o_m, l_m, s_m = h_off[:m].astype(np.uint64), h_len[:m].astype(np.uint64), h_sz[:m]
    simd_keys = orc.fast_cas_keys(host, o_m, l_m, s_m, threads=THREADS)
    reps_cpu, t0 = 0, time.perf_counter()
    while reps_cpu < 1 or time.perf_counter() - t0 < 10.0:
        orc.fast_cas_keys(host, o_m, l_m, s_m, threads=THREADS)
        reps_cpu += 1
    cpu_mt = (time.perf_counter() - t0) / reps_cpu
    t0 = time.perf_counter()
    orc.fast_cas_keys(host, o_m[:4000], l_m[:4000], s_m[:4000], threads=1)
    cpu_simd1 = (time.perf_counter() - t0) / 4000
    emit({"config": 2, "files": n, "message_bytes": msg_bytes, "compressions": comps,
          "k2_ms": t * 1e3, "files_per_s": n / t, "hashed_gb_per_s": msg_bytes / t / 1e9,
          "valu_slot_frac": comps * 1014 / 64 / t / (1024 * 2.4e9 / 2),
          "hbm_frac": msg_bytes / t / 8e12, "parity_sample": ok,
          "cpu_simd_parity_vs_gpu": bool((simd_keys == k[:m]).all()),
          "cpu_scalar_1thread_files_per_s": 1 / cpu1,
          "cpu_simd_1thread_files_per_s": 1 / cpu_simd1,
          "cpu_simd_all_cores_files_per_s": m / cpu_mt,
          "cpu_sample": f"first {m} files of the arena, {reps_cpu} passes", "cores": THREADS})


def config3e(eng, orc, n: int, batch: int):
    pinned = eng.alloc_pinned(n * 57344)
    try:
        rng = np.random.default_rng(3)
        chunk = 1 << 26
        for o in range(0, n * 57344, chunk):
            m = min(chunk, n * 57344 - o)
            pinned[o:o + m] = rng.integers(0, 256, m, dtype=np.uint8)
        sizes = rng.integers(102401, 2 ** 40, n, dtype=np.uint64)
        eng.hash_sampled_host(pinned[: 1024 * 57344], sizes[:1024], batch_files=batch)
        t = time.perf_counter()
        keys = eng.hash_sampled_host(pinned, sizes, batch_files=batch)
        dt = time.perf_counter() - t
        m = 4096
        ok = bool((orc.fast_cas_keys_strided(pinned[: m * 57344], 57344, 57344, sizes[:m], THREADS)
                   == keys[:m]).all())
        emit({"config": "3-e2e", "files": n, "batch_files": batch, "seconds": dt,
              "files_per_s": n / dt, "h2d_gb_per_s": n * 57344 / dt / 1e9,
              "hashed_gb_per_s": n * 57352 / dt / 1e9, "parity_first_4096": ok,
              "note": "PCIe-inclusive: pinned host -> HBM on a side stream, overlapped with K1"})
    finally:
        eng.free_pinned(pinned)


def config4(eng, orc, n_total: int, batch: int, dup: int, shards: int = 1):
    """One rank's share of the 100M-file / 8-GPU library (12.5M files): hash in resident
    batches of `batch` files (content regenerated per batch on the device, untimed), keep
    all keys, then group all of them (K4h/K5h: bucket partition + LDS hash min).  Grouping is checked against the
    generator's duplicate truth for every file."""
    import torch
    content = torch.empty((batch, 57344), dtype=torch.uint8, device="cuda")
    sizes = torch.empty(batch, dtype=torch.int64, device="cuda")
    keys = torch.empty(n_total, dtype=torch.int64, device="cuda")
    hash_s = 0.0
    for f0 in range(0, n_total, batch):
        m = min(batch, n_total - f0)
        eng.synth_sampled(44, f0, m, content, sizes, 57344, dup_permille=dup)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        eng.hash_sampled(content, sizes, keys[f0:f0 + m], n=m)
        b.record()
        torch.cuda.synchronize()
        hash_s += a.elapsed_time(b) / 1e3
    del content
    rep = torch.empty(n_total, dtype=torch.int32, device="cuda")
    eng.group(keys, rep)  # warm (workspace)
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        eng.group(keys, rep, want_objects=False)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 1e3)
    gs = float(np.median(ts))
    objects = eng.group(keys, rep)
    roots = torch.empty(n_total, dtype=torch.int64, device="cuda")
    eng.synth_roots(44, 0, n_total, roots, dup_permille=dup)
    r = roots.cpu().numpy()
    uniq, inv = np.unique(r, return_inverse=True)
    first = np.full(len(uniq), n_total, dtype=np.int64)
    np.minimum.at(first, inv, np.arange(n_total))
    ok = objects == len(uniq) and bool((rep.cpu().numpy() == first[inv]).all())
    del roots, r, inv, first
    # grouping algorithmic bytes per key (bench.group_bytes_per_key): 36 up to 1,441,792 keys
    # (the region chain), 68 up to 40 M (two-level region chain), 76 above (the partition chain)
    bpk = 36 if n_total <= 256 * 5632 else (68 if n_total <= 40_000_000 else 76)
    out = {"config": "4-rank-share" if n_total < 100_000_000 else "4-full-library",
           "files": n_total, "dup_permille": dup,
           "hash_kernel_s": hash_s, "hash_files_per_s": n_total / hash_s,
           "group_s": gs, "group_keys_per_s": n_total / gs, "group_bytes_per_key": bpk,
           "group_hbm_gb_per_s_algorithmic": bpk * n_total / gs / 1e9,
           "group_hbm_frac": bpk * n_total / gs / 1e9 / 8000.0, "objects": objects,
           "grouping_equals_duplicate_truth": ok}
    if shards > 1:
        # the multi-GPU key-range exchange path, all shards on this device (peer copies are
        # device-local here): rep of every file == the local grouping's
        from spacedrive_amd.multi import MultiEngine
        me = MultiEngine([0] * shards)
        cuts = [n_total * i // shards for i in range(shards + 1)]
        parts = [keys[cuts[i]:cuts[i + 1]] for i in range(shards)]
        me.group(parts, cuts[:-1])  # warm
        t = time.perf_counter()
        reps, mobjects = me.group(parts, cuts[:-1])
        torch.cuda.synchronize()
        out["multi_group_shards"] = shards
        out["multi_group_s_one_device"] = time.perf_counter() - t
        out["multi_group_equals_local"] = mobjects == objects and all(
            bool(torch.equal(reps[i], rep[cuts[i]:cuts[i + 1]])) for i in range(shards))
        del reps
        me.close()
    emit(out)


def config5(eng, orc, gib: float, file_mb: int):
    """Validator (file_checksum, validation/hash.rs:11-25) at BASELINE size: (a) one 64 GiB
    resident buffer, (b) 64 GiB as 16 resident multi-GiB files (4 GiB each), every digest
    verified IN FULL against the oracle's tree-parallel CPU hash of the same generated
    stream, (c) a streamed file_checksum of a multi-GiB tmpfs file."""
    import torch
    n = int(gib * (1 << 30))
    buf = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    eng.synth_stream(5, 0, 0, n, buf)
    torch.cuda.synchronize()
    eng.checksum_dev(buf, min(n, 1 << 30))
    t = time.perf_counter()
    digest = eng.checksum_dev(buf, n)
    dt = time.perf_counter() - t
    t = time.perf_counter()
    want = orc.stream_blake3_mt(5, 0, n, THREADS).hex()
    cpu_mt = time.perf_counter() - t
    comps = n // 64 + n // 1024
    emit({"config": 5, "bytes": n, "seconds": dt, "gb_per_s": n / dt / 1e9, "digest": digest,
          "valu_slot_frac": comps * 1014 / 64 / dt / (1024 * 2.4e9 / 2),
          "spec_op_frac": comps * 792 / dt / 78.6432e12, "hbm_frac": n / dt / 8e12,
          "parity_full": digest == want, "cpu_tree_parallel_gb_per_s": n / cpu_mt / 1e9,
          "cpu_threads": THREADS})
    # (b) 16 multi-GiB files of the same 64 GiB, each its own stream and its own digest
    nf = 16
    fl = n // nf
    ts, digs = [], []
    for f in range(nf):
        eng.synth_stream(5, 100 + f, 0, fl, buf[f * fl:])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for f in range(nf):
        digs.append(eng.checksum_dev(buf[f * fl:], fl))
    dtf = time.perf_counter() - t
    wants = [orc.stream_blake3_mt(5, 100 + f, fl, THREADS).hex() for f in range(nf)]
    ok = digs == wants
    emit({"config": "5-files", "files": nf, "file_bytes": fl, "bytes": nf * fl, "seconds": dtf,
          "gb_per_s": nf * fl / dtf / 1e9, "hbm_frac": nf * fl / dtf / 8e12, "parity_full": ok})
    # (b') the same 16 files in ONE launch chain (sd_cas_checksums_dev, K3b: the validator
    # job's batch form), HIP events on the stream
    import numpy as np
    offs = torch.tensor([f * fl for f in range(nf)], dtype=torch.int64, device="cuda")
    lens = torch.full((nf,), fl, dtype=torch.int64, device="cuda")
    out = torch.zeros((nf, 32), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    eng.checksums_dev(buf, offs, lens, out, stream=s.cuda_stream)
    tb = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        eng.checksums_dev(buf, offs, lens, out, stream=s.cuda_stream)
        b.record(s)
        b.synchronize()
        tb.append(a.elapsed_time(b) / 1e3)
    dtb = float(np.median(tb))
    okb = [bytes(r).hex() for r in out.cpu().numpy()] == wants
    emit({"config": "5-files-batch", "files": nf, "bytes": nf * fl, "seconds": dtb,
          "gb_per_s": nf * fl / dtb / 1e9, "hbm_frac": nf * fl / dtb / 8e12, "parity_full": okb})
    del buf
    torch.cuda.empty_cache()
    # (c) streamed file_checksum through pinned staging (tmpfs file)
    path = "/dev/shm/sdcas_validator.bin"
    L = file_mb << 20
    try:
        with open(path, "wb") as fh:
            for off in range(0, L, 256 << 20):
                fh.write(orc.fill_content_range(6, 0, off, min(256 << 20, L - off)).tobytes())
        eng.file_checksum(path)
        t = time.perf_counter()
        h = eng.file_checksum(path)
        dt = time.perf_counter() - t
        t = time.perf_counter()
        w1 = orc.file_checksum(path)
        cpu1 = time.perf_counter() - t
        t = time.perf_counter()
        wm = orc.file_checksum_mt(path, THREADS)
        cpum = time.perf_counter() - t
        official = None
        try:  # hash.rs's loop with the BLAKE3 team's C library (the crate's speed, 1 thread)
            from oracle.pyoracle import ExtBlake3
            ext = ExtBlake3()
            t = time.perf_counter()
            wo = ext.file_checksum(path)
            official = {"library": f"BLAKE3 C {ext.version()} (libclang-cpp.so)",
                        "cpu_1thread_gb_per_s": L / (time.perf_counter() - t) / 1e9, "parity": wo == h}
        except OSError:
            pass
        emit({"config": "5-file", "bytes": L, "gpu_seconds": dt, "gpu_gb_per_s": L / dt / 1e9,
              "cpu_oracle_1thread_gb_per_s": L / cpu1 / 1e9,
              "cpu_oracle_tree_parallel_gb_per_s": L / cpum / 1e9, "cpu_threads": THREADS,
              "cpu_official_c": official, "parity_full": h == w1 == wm})
    finally:
        if os.path.exists(path):
            os.unlink(path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", action="append", required=True)
    ap.add_argument("--c1-files", type=int, default=10_000)
    ap.add_argument("--c2-files", type=int, default=1_000_000)
    ap.add_argument("--c3-files", type=int, default=200_000)
    ap.add_argument("--c3-batch", type=int, default=32768)
    ap.add_argument("--c4-files", type=int, default=12_500_000)
    ap.add_argument("--c4-batch", type=int, default=1_250_000)
    ap.add_argument("--c5-gib", type=float, default=64.0)
    ap.add_argument("--c5-file-mb", type=int, default=4096)
    a = ap.parse_args()
    import torch  # noqa: F401

    from oracle.pyoracle import Oracle
    from spacedrive_amd import CasEngine
    eng = CasEngine(0)
    orc = Oracle()
    for c in a.config:
        if c == "1":
            config1(eng, orc, a.c1_files, "/dev/shm/sdcas_c1")
        elif c == "2":
            config2(eng, orc, a.c2_files, 5)
        elif c == "3e":
            config3e(eng, orc, a.c3_files, a.c3_batch)
        elif c == "4":
            config4(eng, orc, a.c4_files, a.c4_batch, 300)
        elif c == "4full":
            config4(eng, orc, 100_000_000, a.c4_batch, 300, shards=8)
        elif c == "5":
            config5(eng, orc, a.c5_gib, a.c5_file_mb)


if __name__ == "__main__":
    main()
