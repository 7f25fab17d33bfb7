#!/usr/bin/env python3
"""K3 timing (config 5 shape): BLAKE3 of one device-resident buffer of --gib GiB.

Times sd_cas_checksum_dev (K3 chunk groups + CV reduce levels) with HIP events on the
engine's stream; prints one JSON line with the digest so A/B builds (SD_HIP_CAS_LIB) can
be checked against each other, and the oracle digest of a --check-mib prefix.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=64.0)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--check-mib", type=int, default=64)
    a = ap.parse_args()
    import numpy as np
    import torch
    from spacedrive_amd import CasEngine
    from oracle.pyoracle import Oracle
    eng = CasEngine(0)
    n = int(a.gib * (1 << 30))
    buf = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    files = n // 57344
    sz = torch.empty(max(files, 1), dtype=torch.int64, device="cuda")
    eng.synth_sampled(5, 0, files, buf, sz, 57344)
    buf[files * 57344:].zero_()
    torch.cuda.synchronize()
    eng.checksum_dev(buf, n)
    ts = []
    for _ in range(a.iters):
        t = time.perf_counter()
        d = eng.checksum_dev(buf, n)
        ts.append(time.perf_counter() - t)
    dt = float(np.median(ts))
    pre = a.check_mib << 20
    ok = eng.checksum_dev(buf, pre) == Oracle().blake3(buf[:pre].cpu().numpy().tobytes()).hex()
    comps = n // 64 + n // 1024
    print(json.dumps({"lib": os.path.basename(os.environ.get("SD_HIP_CAS_LIB", "in-tree")),
                      "bytes": n, "ms": dt * 1e3, "ms_all": [x * 1e3 for x in ts],
                      "gb_per_s": n / dt / 1e9,
                      "valu_slot_frac": comps * 1014 / 64 / dt / (1024 * 2.4e9 / 2),
                      "digest": d, "parity_prefix": ok}), flush=True)


if __name__ == "__main__":
    main()
