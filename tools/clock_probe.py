#!/usr/bin/env python3
"""Socket power and shader clock while one kernel runs back to back (DESIGN.md §8 item 2:
why K2 and the validator's lane kernel run at a lower clock than K1).  For each workload
the kernel is launched in a loop for --seconds on the engine's stream while this process
samples `rocm-smi -P -g --json` (a child process; it reads the SMI, no HIP) every ~0.2 s;
prints one JSON line per workload with the median power and sclk over the samples taken
after a 1 s settle, and the kernel's own rate.
  k1     K1 (sd_cas_sampled_kernel) on 1,310,720 synthetic sampled files (the bench batch)
  k1c    the same kernel on CONSTANT content (all-zero bytes): the data-toggle share of power
  k2     K2 on config 2's 1 M whole-file messages (sizes U(1, 102,400))
  k2c    the same messages with all-zero content
  lane   the validator on 1 M buffers of U(0, 16) KiB (the lane-per-buffer kernel)
  k1g    the fused chain (K1G + the region tables: the bench's N = 1 step)
  one    the validator's K3 on one 16 GiB buffer
"""
import argparse
import json
import os
import re
import subprocess
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def smi_sample():
    """(power W, sclk MHz) from rocm-smi's JSON, or (None, None)."""
    try:
        r = subprocess.run(["rocm-smi", "-P", "-g", "--json"], capture_output=True, text=True, timeout=10)
        d = json.loads(r.stdout)
    except (OSError, ValueError, subprocess.SubprocessError):
        return None, None
    card = next(iter(v for k, v in d.items() if k.startswith("card")), {})
    power = sclk = None
    for k, v in card.items():
        kl = k.lower()
        if "power" in kl and power is None:
            m = re.search(r"[\d.]+", str(v))
            power = float(m.group()) if m else None
        if "sclk" in kl and sclk is None:
            m = re.search(r"(\d+)\s*mhz", str(v).lower())
            sclk = float(m.group(1)) if m else None
    return power, sclk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("workloads", nargs="*", default=["k1", "k1c", "k2", "k2c", "lane"])
    a = ap.parse_args()
    import numpy as np
    import torch
    from spacedrive_amd import CasEngine
    eng = CasEngine(0)
    print(json.dumps({"idle_smi": smi_sample()}), flush=True)
    for w in a.workloads:
        torch.cuda.empty_cache()
        if w in ("k1", "k1c"):
            F = 1_310_720
            content = torch.empty((F, 57344), dtype=torch.uint8, device="cuda")
            sizes = torch.empty(F, dtype=torch.int64, device="cuda")
            keys = torch.empty(F, dtype=torch.int64, device="cuda")
            eng.synth_sampled(3, 0, F, content, sizes, 57344)
            if w == "k1c":
                content.zero_()
            units, unit = F, "files"
            launch = lambda: eng.hash_sampled(content, sizes, keys)  # noqa: E731
        elif w == "k1g":
            F = 1_310_720
            content = torch.empty((F, 57344), dtype=torch.uint8, device="cuda")
            sizes = torch.empty(F, dtype=torch.int64, device="cuda")
            keys = torch.empty(F, dtype=torch.int64, device="cuda")
            rep = torch.empty(F, dtype=torch.int32, device="cuda")
            ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
            eng.synth_sampled(3, 0, F, content, sizes, 57344, dup_permille=300)
            units, unit = F, "files"
            launch = lambda: eng.hash_group_sampled(content, sizes, keys, rep, ovf, want_objects=False)  # noqa: E731
        elif w == "one":
            n = 16 << 30
            arena = torch.empty(n, dtype=torch.uint8, device="cuda")
            eng.synth_stream(77, 0, 0, n, arena)
            units, unit = n, "bytes"
            launch = lambda: eng.checksum_dev(arena)  # noqa: E731  (blocking: returns the hex)
        elif w in ("k2", "k2c"):
            n = 1_000_000
            sizes = torch.empty(n, dtype=torch.int64, device="cuda")
            lens = torch.empty(n, dtype=torch.int32, device="cuda")
            offs = torch.empty(n, dtype=torch.int64, device="cuda")
            nbytes = eng.synth_small(11, 0, n, sizes, lens, offs, None)
            arena = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
            eng.synth_small(11, 0, n, sizes, lens, offs, arena)
            if w == "k2c":
                arena.zero_()
            keys = torch.empty(n, dtype=torch.int64, device="cuda")
            units, unit = n, "files"
            launch = lambda: eng.hash_packed(arena, offs, lens, sizes, keys)  # noqa: E731
        elif w == "lane":
            n = 1 << 20
            rng = np.random.default_rng(5)
            ln = rng.integers(0, (16 << 10) + 1, n, dtype=np.uint64)
            of = np.zeros(n, dtype=np.uint64)
            of[1:] = np.cumsum((ln[:-1] + 127) // 128 * 128)
            ab = (int(of[-1] + ln[-1]) + 127) // 128 * 128 + 128
            arena = torch.empty(ab, dtype=torch.uint8, device="cuda")
            eng.synth_stream(77, 0, 0, ab // 8 * 8, arena)
            d_offs = torch.from_numpy(of.view(np.int64)).cuda()
            d_lens = torch.from_numpy(ln.view(np.int64)).cuda()
            out = torch.zeros((n, 32), dtype=torch.uint8, device="cuda")
            units, unit = n, "buffers"
            launch = lambda: eng.checksums_dev(arena, d_offs, d_lens, out)  # noqa: E731
        else:
            raise SystemExit(f"unknown workload {w}")
        torch.cuda.synchronize()
        launch()
        torch.cuda.synchronize()
        stop = threading.Event()
        count = [0]

        def loop():
            torch.cuda.set_device(0)
            while not stop.is_set():
                launch()
                torch.cuda.synchronize()
                count[0] += 1
        th = threading.Thread(target=loop)
        t0 = time.time()
        th.start()
        samples = []
        while time.time() - t0 < a.seconds:
            time.sleep(0.2)
            p, c = smi_sample()
            samples.append((time.time() - t0, p, c))
        stop.set()
        th.join()
        dt = time.time() - t0
        settled = [s for s in samples if s[0] > 1.0]
        pw = [s[1] for s in settled if s[1] is not None]
        ck = [s[2] for s in settled if s[2] is not None]
        print(json.dumps({"workload": w, "launches": count[0], "seconds": round(dt, 2),
                          f"{unit}_per_s": units * count[0] / dt,
                          "power_w_median": float(np.median(pw)) if pw else None,
                          "sclk_mhz_median": float(np.median(ck)) if ck else None,
                          "samples": len(settled)}), flush=True)
        del launch
        content = sizes = keys = lens = offs = arena = d_offs = d_lens = out = rep = ovf = None  # noqa: F841
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
