#!/usr/bin/env python3
"""Config 1 A/B: the 10k-file tmpfs library of tools/bench_configs.py config 1, the GPU
drop-in (sd_cas_generate_cas_ids_from_paths) timed 7x and the CPU oracle (16-thread gather +
AVX-512 hash) 5x, medians; keys checked against each other.  One JSON line."""
import json
import math
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

THREADS = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)


def main():
    import torch  # noqa: F401
    from oracle.pyoracle import Oracle
    from spacedrive_amd import CasEngine
    eng, orc = CasEngine(0), Oracle()
    n_files, root = 10_000, "/dev/shm/sdcas_ab1"
    rng = np.random.default_rng(1)
    sizes = np.exp(rng.uniform(math.log(1024), math.log(10 * 1024 * 1024), n_files)).astype(np.int64)
    os.makedirs(root, exist_ok=True)
    paths = []
    try:
        for i, s in enumerate(sizes):
            p = os.path.join(root, f"f{i:05d}")
            with open(p, "wb") as fh:
                fh.write(rng.integers(0, 256, int(s), dtype=np.uint8).tobytes())
            paths.append(p)
        keys, errs = eng.generate_cas_keys_from_paths(paths, sizes)
        assert not errs.any()
        g = []
        for _ in range(7):
            t = time.perf_counter()
            k2, _ = eng.generate_cas_keys_from_paths(paths, sizes)
            g.append(time.perf_counter() - t)
            assert (k2 == keys).all()
        c = []
        for _ in range(5):
            t = time.perf_counter()
            kc, _ = orc.generate_cas_keys_paths(paths, sizes, THREADS, simd=True)
            c.append(time.perf_counter() - t)
        assert (kc == keys).all()
        print(json.dumps({"gpu_ms": [round(x * 1e3, 2) for x in g], "cpu_ms": [round(x * 1e3, 2) for x in c],
                          "gpu_files_per_s_median": n_files / float(np.median(g)),
                          "cpu_files_per_s_median": n_files / float(np.median(c)), "threads": THREADS}), flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
