#!/usr/bin/env python3
"""Where K1's random-content power goes: the ~200 W random content costs
over constant content, split into HBM / fabric traffic and on-chip data toggling, in ONE
gpurun session.  Each variant of tools/ubench_k1 (`sustain <mode> <data> <seconds>`) runs
back to back as a child process while this process samples `rocm-smi -P -g --json`; energy
per file = (median power - idle power) / rate, after a 1 s settle.
  k1_rand / k1_const     K1 on random / constant (0x5a) content, loads from HBM (the product)
  l2_rand / l2_const     the same lane program, every lane's loads aimed at a 32-file window
                         (L2-resident: no HBM traffic, lanes still hash different data)
  comp_rand / comp_const compute-only, 953 compressions per lane, message evolving / constant
Splits (J per file, dynamic): HBM + fabric beyond L2 = k1_rand - l2_rand; on-chip toggling of
random vs constant data = l2_rand - l2_const; the HBM share of the random-content cost =
(k1_rand - k1_const) - (l2_rand - l2_const).  Two interleaved rounds.  --variants
k1_rand,k1_line_rand,k1_quad_rand: the A/B of a layout with DRAM row locality.
Usage: power_split.py [--seconds S] [--bin tools/ubench_k1]"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from clock_probe import smi_sample  # noqa: E402

VARIANTS = {"k1_rand": (0, 1), "k1_const": (0, 0), "l2_rand": (1, 1), "l2_const": (1, 0),
            "comp_rand": (3, 1), "comp_const": (7, 1),
            # --variants: the HBM-energy A/B — 64-file tiled layouts, so a wave's loads of one
            # iteration hit consecutive lines (DRAM row locality) instead of 64 files' rows
            "k1_line_rand": (5, 1), "k1_quad_rand": (6, 1)}
DEFAULT = ["k1_rand", "k1_const", "l2_rand", "l2_const", "comp_rand", "comp_const"]


def run(binary, name, seconds):
    mode, data = VARIANTS[name]
    t0 = time.time()
    p = subprocess.Popen([binary, "sustain", str(mode), str(data), str(seconds)],
                         stdout=subprocess.PIPE, text=True)
    samples = []
    while p.poll() is None:
        time.sleep(0.2)
        pw, ck = smi_sample()
        samples.append((time.time() - t0, pw, ck))
    out = p.stdout.read()
    if p.returncode != 0:
        raise SystemExit(f"{name}: ubench_k1 exited {p.returncode}: {out}")
    line = json.loads(out.strip().splitlines()[-1])
    # the settle: skip the first 1.5 s (allocation + fill + 1 s of kernels)
    settled = [s for s in samples if s[0] > 1.5 and s[0] < seconds]
    pw = sorted(s[1] for s in settled if s[1] is not None)
    ck = sorted(s[2] for s in settled if s[2] is not None)
    line.update({"variant": name, "power_w_median": pw[len(pw) // 2] if pw else None,
                 "sclk_mhz_median": ck[len(ck) // 2] if ck else None, "samples": len(settled)})
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--bin", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "ubench_k1"))
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", default=",".join(DEFAULT))
    a = ap.parse_args()
    idle = [smi_sample()[0] for _ in range(5)]
    seen = sorted(x for x in idle if x is not None)
    if not seen:
        raise SystemExit("rocm-smi gave no power reading")
    idle_w = seen[len(seen) // 2]
    print(json.dumps({"idle_power_w": idle_w, "idle_samples": idle}), flush=True)
    res = {}
    for r in range(a.rounds):
        for name in a.variants.split(","):
            line = run(a.bin, name, a.seconds)
            line["round"] = r
            print(json.dumps(line), flush=True)
            res.setdefault(name, []).append(line)
    # J per file (dynamic), median over rounds
    e = {}
    for name, lines in res.items():
        vals = sorted((ln["power_w_median"] - idle_w) / ln["files_per_s"] for ln in lines
                      if ln["power_w_median"] and ln["files_per_s"])
        e[name] = vals[len(vals) // 2] if vals else None
    uj = {k: (v * 1e6 if v is not None else None) for k, v in e.items()}
    split = None
    if all(uj.get(k) for k in ("k1_rand", "k1_const", "l2_rand", "l2_const")):
        total = uj["k1_rand"] - uj["k1_const"]
        onchip = uj["l2_rand"] - uj["l2_const"]
        split = {"random_minus_constant_uj_per_file": total,
                 "on_chip_data_toggling_uj_per_file": onchip,
                 "hbm_fabric_data_toggling_uj_per_file": total - onchip,
                 "hbm_fabric_beyond_l2_uj_per_file_random": uj["k1_rand"] - uj["l2_rand"],
                 "hbm_fabric_beyond_l2_uj_per_file_constant": uj["k1_const"] - uj["l2_const"],
                 "compute_only_msg_toggling_uj_per_file": (uj["comp_rand"] - uj["comp_const"])
                 if uj.get("comp_rand") and uj.get("comp_const") else None}
    print(json.dumps({"summary": True, "idle_power_w": idle_w, "dynamic_uj_per_file": uj, "split": split}),
          flush=True)


if __name__ == "__main__":
    main()
