#!/usr/bin/env python3
"""100-file job steps through sd_cas_generate_cas_ids_from_paths (the reference's step
shape, file_identifier/mod.rs:34): 300 steps over sampled and whole files on tmpfs, then
config 1's size mix walked 100 paths at a time over 3,000 files; with
the tracing build (tools/ablib/patch_trace_paths.py) stderr carries per-phase times."""
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def main():
    import torch  # noqa: F401
    from spacedrive_amd import CasEngine
    from oracle.pyoracle import Oracle
    eng = CasEngine(0)
    orc = Oracle()
    rng = np.random.default_rng(3)
    root = "/dev/shm/sdcas_js"
    os.makedirs(root, exist_ok=True)
    try:
        for kind, lo, hi in (("sampled", 200_000, 2_000_000), ("whole", 1_000, 100_000), ("mixed", 1_000, 2_000_000)):
            paths, sizes = [], []
            for i in range(100):
                s = int(np.exp(rng.uniform(np.log(lo), np.log(hi))))
                p = os.path.join(root, f"{kind}{i:03d}")
                with open(p, "wb") as fh:
                    fh.write(rng.integers(0, 256, s, dtype=np.uint8).tobytes())
                paths.append(p)
                sizes.append(s)
            keys, st = eng.generate_cas_keys_from_paths(paths, sizes)
            want = [int(orc.generate_cas_id(p, s), 16) for p, s in zip(paths, sizes)]
            parity = bool(not st.any() and (keys == np.array(want, dtype=np.uint64)).all())
            for _ in range(20):
                eng.generate_cas_keys_from_paths(paths, sizes)
            ts = []
            for _ in range(300):
                t = time.perf_counter()
                eng.generate_cas_keys_from_paths(paths, sizes)
                ts.append(time.perf_counter() - t)
            print(f"{kind}: median {np.median(ts) * 1e3:.3f} ms  p10 {np.percentile(ts, 10) * 1e3:.3f}  p90 {np.percentile(ts, 90) * 1e3:.3f}  parity {parity}", flush=True)
        # config 1's shape (log-uniform 1 KiB..10 MiB) walked 100 paths at a time over 3,000
        # files (~3.4 GB, beyond the host's last-level cache: every step reads new files)
        shutil.rmtree(root, ignore_errors=True)
        os.makedirs(root, exist_ok=True)
        n = int(os.environ.get("SD_JS_C1_FILES", "3000"))
        paths, sizes = [], []
        for i in range(n):
            s = int(np.exp(rng.uniform(np.log(1024), np.log(10 << 20))))
            p = os.path.join(root, f"c1_{i:05d}")
            with open(p, "wb") as fh:
                fh.write(rng.integers(0, 256, s, dtype=np.uint8).tobytes())
            paths.append(p)
            sizes.append(s)
        sizes = np.array(sizes, dtype=np.int64)
        keys, st = eng.generate_cas_keys_from_paths(paths, sizes)
        idx = list(range(0, n, 97))
        want = np.array([int(orc.generate_cas_id(paths[i], int(sizes[i])), 16) for i in idx], dtype=np.uint64)
        parity = bool(not st.any() and (keys[idx] == want).all())
        ts = []
        for rep in range(3):
            for i in range(0, n, 100):
                t = time.perf_counter()
                k, _ = eng.generate_cas_keys_from_paths(paths[i:i + 100], sizes[i:i + 100])
                ts.append(time.perf_counter() - t)
                parity = parity and bool((k == keys[i:i + 100]).all())
        print(f"config1-walk: median {np.median(ts) * 1e3:.3f} ms  mean {np.mean(ts) * 1e3:.3f}  p10 {np.percentile(ts, 10) * 1e3:.3f}  p90 {np.percentile(ts, 90) * 1e3:.3f}  parity {parity}", flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
