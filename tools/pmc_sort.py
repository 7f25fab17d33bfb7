#!/usr/bin/env python3
"""HBM bytes per key of the Object-grouping methods at 12.5 M keys (config 4's rank share)
from the rocprofv3 --pmc passes of tools/gpu_r6_pmc_sort.sh: per method (one process each,
tools/bench_group.py --only hash|lsd|lsdapi, `chain_calls` chains per process), the
FETCH_SIZE / WRITE_SIZE of every sd_* dispatch summed and divided by chain_calls x keys.
gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE reports half the bytes of
a wide coalesced read, so it is doubled; both are in KiB.  Algorithmic bytes per key (ALGO
below): hash chain 68 B (bench.group_bytes_per_key, two-level region chain); the LSD sort as
implemented (group.hip): 8 passes x (upsweep reads the 8-B key + scatter reads and writes key
+ 4-B idx = 32 B), then the runs kernel; SURVEY §8(d)'s model of a sort without a separate
histogram read (8 x 24 + 16 = 208 B) is reported beside it.
Usage: pmc_sort.py <out dir>   (expects <out>/<method>_{fetch,write,hit}/ and *.log)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KEYS = 12_500_000
# round 6: "lsd" = the product's LSD grouping (sd_cas_group_dev, SD_CAS_GROUP_SORT): 8 passes x
# 32 B + rep[i] = i laid down by the first pass (4) + the runs kernel reading the sorted pairs
# (12) + one 4-B rep store per key that is not its run's head ((n - objects) / n x 4, added
# below); "lsdapi" = sd_cas_sort_pairs_dev + sd_cas_group_sorted_dev (every rep stored: 272)
ALGO = {"hash": 68, "lsd": 8 * 32 + 4 + 12, "lsdapi": 8 * 32 + 12 + 4}
SURVEY_MODEL = {"hash": None, "lsd": 208, "lsdapi": 208}
METHODS = ("hash", "lsd", "lsdapi")


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
    for m in METHODS:
        if not os.path.exists(os.path.join(out, f"{m}_fetch.log")):
            continue
        chains, objects = None, None
        with open(os.path.join(out, f"{m}_fetch.log")) as fh:
            for line in fh:
                if line.startswith("{"):
                    chains = json.loads(line)["chain_calls"]
                    objects = json.loads(line).get("objects")
        algo = ALGO[m] + (4 * (KEYS - objects) / KEYS if m == "lsd" and objects else 0)
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
                  "write_b_per_key": tot_w, "algorithmic_b_per_key": algo,
                  "measured_over_algorithmic": (tot_r + tot_w) / algo,
                  "survey_model_b_per_key": SURVEY_MODEL[m], "kernels": per_kernel}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
