#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel over every *counter_collection.csv
under the given directories; prints one JSON object {kernel: {counter: mean, calls: n}}."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"calls": max(len(v) for v in cs.values())}
           for k, cs in acc.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
