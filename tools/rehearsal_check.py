#!/usr/bin/env python3
"""Checks a one-GPU rehearsal of the N-GPU bench line (SD_BENCH_ONE_DEVICE=1 bench.py --gpus N,
VERDICT r5 #3): pulls the JSON line out of the log (gloo's connection chatter surrounds it) and
checks what the driver's N-GPU run will need — n_gpus N, the G-specific exchange slot sizes,
no timed step overflowed its fixed capacity, no host sync per step, and non-null roofline /
group / cpu_baseline / e2e with e2e parity.  Prints one JSON summary (and writes the bare line
next to the log as <log>.json).  Usage: rehearsal_check.py <log> <N>"""
import json
import sys


def find(d, key):
    """The first value of `key` anywhere in the nested line."""
    if isinstance(d, dict):
        if key in d:
            return d[key]
        for v in d.values():
            r = find(v, key)
            if r is not None:
                return r
    return None


def main():
    path, n = sys.argv[1], int(sys.argv[2])
    line = None
    for raw in open(path, errors="replace"):
        i = raw.find('{"metric"')
        if i >= 0:
            line = json.loads(raw[i:])
    if line is None:
        raise SystemExit(f"{path}: no bench line")
    out = path.rsplit(".", 1)[0] + (".line.json" if path.endswith(".json") else ".json")
    with open(out, "w") as fh:
        json.dump(line, fh, indent=1)
    e2e = line.get("e2e") or {}
    checks = {
        "n_gpus": line.get("n_gpus") == n,
        "capacity_per_peer": find(line, "capacity_per_peer") is not None,
        "timed_steps_overflowed_0": find(line, "timed_steps_overflowed") == 0,
        "host_syncs_per_step_0": find(line, "host_syncs_per_step") == 0,
        "roofline": line.get("roofline") is not None,
        "group": line.get("group") is not None,
        "cpu_baseline": line.get("cpu_baseline") is not None,
        "e2e": bool(e2e),
        "e2e_parity": e2e.get("parity_vs_resident_k1") is True,
    }
    print(json.dumps({"log": path, "n_gpus": line.get("n_gpus"), "value": line.get("value"),
                      "capacity_per_peer": find(line, "capacity_per_peer"),
                      "spill_per_peer": find(line, "spill_per_peer"), "checks": checks,
                      "ok": all(checks.values())}))
    if not all(checks.values()):
        sys.exit(1)


if __name__ == "__main__":
    main()
