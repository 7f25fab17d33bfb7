#!/usr/bin/env python3
"""VALU busy per kernel from the rocprofv3 --pmc passes of tools/pmc_valu.sh.

Counter conventions (MI355X_MICROARCH.md, rocprofv3 PMC section): rocprofv3 reports
GRBM_GUI_ACTIVE summed over the 8 XCDs, so the kernel's wall clock in shader cycles is
GRBM_GUI_ACTIVE / 8; SQ_ACTIVE_INST_VALU is summed over every wave and counts quad-cycles;
the chip has 256 CUs x 4 SIMDs = 1,024 SIMDs.
  valu_busy            = SQ_ACTIVE_INST_VALU x 4 / (1,024 x GRBM_GUI_ACTIVE / 8) — rocprof's
                         VALUBusy (the gfx94x formula ROCm 7.2 falls back to on gfx950); it
                         charges every VALU instruction one quad-cycle (4 cycles)
  valu_busy_full_rate  = SQ_INSTS_VALU x 2 / (1,024 x GRBM_GUI_ACTIVE / 8) — the same with
                         every wave64 instruction at the full SIMD32 rate (2 cycles): a floor
  clock_ghz            = GRBM_GUI_ACTIVE / 8 / the kernel's mean duration (kernel trace)
  instr_rate_t_per_s   = SQ_INSTS_VALU x 64 lanes / the kernel's mean duration (T lane-instr/s:
                         the achieved integer instruction rate, vs the 78.6 T full-rate peak)
Prints one JSON object {kernel: {...}} (per-dispatch means)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4


def summarize(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9)
    out = {}
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "GRBM_GUI_ACTIVE" not in m or "SQ_INSTS_VALU" not in m:
            continue
        wall = m["GRBM_GUI_ACTIVE"] / 8
        rec = {"dispatches": max(len(v) for v in cs.values()), "counters_mean": m,
               "wall_cycles": wall,
               "valu_busy": m.get("SQ_ACTIVE_INST_VALU", 0) * 4 / (SIMDS * wall),
               "valu_busy_full_rate": m["SQ_INSTS_VALU"] * 2 / (SIMDS * wall),
               "valu_instr_per_wave": m["SQ_INSTS_VALU"] / max(m.get("SQ_WAVES", 1), 1)}
        if dur.get(k):
            t = sum(dur[k]) / len(dur[k])
            rec["mean_s"] = t
            rec["clock_ghz"] = wall / t / 1e9
            rec["instr_rate_t_per_s"] = m["SQ_INSTS_VALU"] * 64 / t / 1e12
        out[k] = rec
    return out


def main():
    print(json.dumps(summarize(sys.argv[1:]), indent=1))


if __name__ == "__main__":
    main()
