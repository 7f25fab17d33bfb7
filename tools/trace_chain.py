#!/usr/bin/env python3
"""Per-dispatch breakdown of the grouping launch chains in a rocprofv3 kernel-trace csv:
one block per chain (from the first totals/hist kernel to the bucket_min kernel)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
seq = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:34], r["Grid_Size_X"],
              r["VGPR_Count"]) for r in rows)
chains, i = [], 0
while i < len(seq):
    if seq[i][2].startswith(("sd_part_hist_mix", "sd_part_totals_mix")):
        j = i
        while j < len(seq) and not seq[j][2].startswith("sd_bucket_min"):
            j += 1
        k0 = i - 1 if i and seq[i - 1][2].startswith("__amd_rocclr_fill") else i
        chains.append(seq[k0:j + 1])
        i = j + 1
    else:
        i += 1
for ch in chains[-int(sys.argv[2]) if len(sys.argv) > 2 else 0:]:
    print(f"chain: {(ch[-1][1] - ch[0][0]) / 1e3:.1f} us, {len(ch)} dispatches")
    prev = None
    for c in ch:
        gap = (c[0] - prev) / 1e3 if prev else 0.0
        print(f"  {c[2]:34s} {(c[1] - c[0]) / 1e3:7.1f} us  gap {gap:5.1f}  grid={c[3]} vgpr={c[4]}")
        prev = c[1]
