#!/usr/bin/env python3
"""Combine one gpurun session's VALU / power evidence into profiles/r05_valu_power.json
(read by bench.py into roofline.valu_busy / roofline.power).  Inputs, all from the SAME box
and session (tools/gpu_r5_valu_power.sh):
  <out>/ubench_k1.log   tools/ubench_k1: the compute-only loop of K1's instruction stream
                        (953 compressions per lane, no loads) with its clock from
                        s_memtime / s_memrealtime -> files per shader cycle (clock-free)
  <out>/clock.jsonl     tools/clock_probe.py k1 k1c k1g: kernel rate, rocm-smi power and
                        sclk while the kernel runs back to back (random / all-zero content)
  <out>/p*/             rocprofv3 --kernel-trace --pmc passes (tools/pmc_valu.py)
Usage: valu_power.py <out dir> <session id>"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_valu import summarize  # noqa: E402

N_FILES = 1310720  # ubench_k1's batch (= the bench batch)


def main():
    out, session = sys.argv[1], sys.argv[2]
    best = None
    with open(os.path.join(out, "ubench_k1.log")) as fh:
        for line in fh:
            m = re.match(r"compress-only x953\s+([\d.]+) ms\s+([\d.]+) M files/s\s+clock ([\d.]+) GHz", line)
            if m:
                ms, ghz = float(m.group(1)), float(m.group(3))
                fpc = N_FILES / (ms * 1e-3 * ghz * 1e9)
                if best is None or fpc > best["files_per_cycle"]:
                    best = {"ms": ms, "clock_ghz": ghz, "files_per_cycle": fpc,
                            "files_per_s": N_FILES / (ms * 1e-3)}
    probe = {}
    with open(os.path.join(out, "clock.jsonl")) as fh:
        for line in fh:
            r = json.loads(line)
            if r.get("workload"):
                probe[r["workload"]] = r
    ceiling = {"compute_only": best, "files_per_cycle": best["files_per_cycle"] if best else None}
    if best:
        for w in ("k1", "k1g"):
            r = probe.get(w)
            if r and r.get("sclk_mhz_median"):
                cap = best["files_per_cycle"] * r["sclk_mhz_median"] * 1e6
                ceiling[f"{w}_ceiling_files_per_s_at_capped_clock"] = cap
                ceiling[f"{w}_frac_of_capped_ceiling"] = r["files_per_s"] / cap
        ceiling["k1_frac_of_capped_ceiling"] = ceiling.get("k1g_frac_of_capped_ceiling",
                                                           ceiling.get("k1_frac_of_capped_ceiling"))
    dirs = sorted(os.path.join(out, d) for d in os.listdir(out) if re.match(r"p\d+$", d))
    rec = {"session": session,
           "method": "one gpurun session: tools/ubench_k1 (compute-only ceiling, in-kernel clock), "
                     "tools/clock_probe.py (rocm-smi while the kernel loops), rocprofv3 --kernel-trace "
                     "--pmc (tools/pmc_valu.py counter conventions)",
           "ceiling": ceiling, "clock_probe": probe, "pmc": summarize(dirs)}
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
