#!/usr/bin/env python3
"""HBM bytes per key of the two Object-grouping methods at 12.5 M keys (config 4's rank share)
from the rocprofv3 --pmc passes of tools/gpu_r5_pmc_sort.sh: per method (one process each,
tools/bench_group.py --only hash|lsd, `chain_calls` chains per process), the FETCH_SIZE /
WRITE_SIZE of every sd_* dispatch summed and divided by chain_calls x keys.  gfx950
correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE reports half the bytes of a wide
coalesced read, so it is doubled; both are in KiB.  Algorithmic bytes per key: hash chain
68 B (bench.group_bytes_per_key, two-level region chain); LSD sort as implemented (group.hip):
8 passes x (upsweep reads the 8-B key + scatter reads and writes key + 4-B idx = 32 B) +
run heads (read 8) + emit (read 12, write the 4-B rep) = 280 B; SURVEY §8(d)'s model of a
sort without a separate histogram read (8 x 24 + 16 = 208 B) is reported beside it.
Usage: pmc_sort.py <out dir>   (expects <out>/{hash,lsd}_{fetch,write,hit}/ and *.log)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KEYS = 12_500_000
ALGO = {"hash": 68, "lsd": 8 * 32 + 8 + 16}
SURVEY_MODEL = {"hash": None, "lsd": 208}


def counters(d):
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not k.startswith("sd_"):
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k][r["Counter_Name"]] += 1
    return acc, calls


def main():
    out = sys.argv[1]
    res = {"keys": KEYS, "correction": "FETCH_SIZE x 2 (gfx950), KiB -> bytes x 1024"}
    for m in ("hash", "lsd"):
        chains = None
        with open(os.path.join(out, f"{m}_fetch.log")) as fh:
            for line in fh:
                if line.startswith("{"):
                    chains = json.loads(line)["chain_calls"]
        fetch, fc = counters(os.path.join(out, f"{m}_fetch"))
        write, _ = counters(os.path.join(out, f"{m}_write"))
        hit, _ = counters(os.path.join(out, f"{m}_hit"))
        per_kernel = {}
        tot_r = tot_w = 0.0
        for k in sorted(set(fetch) | set(write)):
            r = 2 * fetch.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 / (chains * KEYS)
            w = write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024 / (chains * KEYS)
            h = hit.get(k, {})
            hr = h.get("TCC_HIT_sum", 0.0) / max(h.get("TCC_HIT_sum", 0.0) + h.get("TCC_MISS_sum", 0.0), 1.0)
            per_kernel[k] = {"read_b_per_key": r, "write_b_per_key": w, "l2_hit": hr,
                             "dispatches": max(fc.get(k, {}).values() or [0])}
            tot_r += r
            tot_w += w
        res[m] = {"chain_calls": chains, "measured_b_per_key": tot_r + tot_w, "read_b_per_key": tot_r,
                  "write_b_per_key": tot_w, "algorithmic_b_per_key": ALGO[m],
                  "measured_over_algorithmic": (tot_r + tot_w) / ALGO[m],
                  "survey_model_b_per_key": SURVEY_MODEL[m], "kernels": per_kernel}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
