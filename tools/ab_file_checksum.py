#!/usr/bin/env python3
"""Streamed file_checksum A/B: a 4 GiB tmpfs file (oracle content generator), timed 5x per
build; digest checked against the oracle's tree-parallel file hash.  One JSON line."""
import json
import os
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
    L = int(os.environ.get("AB_FILE_BYTES", str(4 << 30))) + 4321
    path = "/dev/shm/sdcas_abfc.bin"
    try:
        with open(path, "wb") as fh:
            for off in range(0, L, 256 << 20):
                fh.write(orc.fill_content_range(6, 0, off, min(256 << 20, L - off)).tobytes())
        h = eng.file_checksum(path)
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            assert eng.file_checksum(path) == h
            ts.append(time.perf_counter() - t)
        ok = h == orc.file_checksum_mt(path, THREADS)
        print(json.dumps({"bytes": L, "ms": [round(x * 1e3, 1) for x in ts],
                          "gb_per_s_median": L / float(np.median(ts)) / 1e9, "parity_full": ok}), flush=True)
    finally:
        if os.path.exists(path):
            os.unlink(path)


if __name__ == "__main__":
    main()
