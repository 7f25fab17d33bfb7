#!/usr/bin/env python3
"""Randomised parity stress for the Object-link emission (sd_cas_identifier_links_ex[_dev],
round 5): for --seconds, draw random jobs and check the device decisions row for row.
  * small jobs (n <= 2,500): against the literal DB replay
    (tests/golden/make_golden.py::replay_identifier_job) — per-step counts, steps, owners,
    actions — through the device AND the host entry point;
  * large jobs (up to 4 M rows): against a numpy closed form (the per-key prefix minimum over
    steps of the Objects rows already hold, seeds, the key's first row) on top of an O(n)
    cursor walk of the reference's orphan query.
Each job draws: chunk 1..300; a key pattern (uniform with duplicates, a few hot keys, small
integers); NO_CAS / ERROR rows (some at chunk ends, so the cursor re-queries them); seeded
Objects (0-40 % of keys, several ids per key, ids in any order); rows that already own an
Object (0-60 %, ids interleaved with the seeds', hot keys owning Objects in many steps).
Prints one JSON line per job and a summary; exits non-zero on the first mismatch."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

NONE = 0xFFFFFFFF


def draw_job(rng, n):
    chunk = int(rng.choice([1, 2, 7, 100, int(rng.integers(1, 300))]))
    pat = rng.choice(["uniform", "hot", "small"])
    if pat == "uniform":
        pool = rng.integers(1, 2 ** 64, max(1, n // int(rng.integers(1, 6))), dtype=np.uint64)
        keys = pool[rng.integers(0, len(pool), n)]
    elif pat == "hot":
        keys = rng.integers(1, 2 ** 64, n, dtype=np.uint64)
        hot = rng.integers(1, 2 ** 64, int(rng.integers(1, 8)), dtype=np.uint64)
        m = rng.random(n) < rng.uniform(0.05, 0.5)
        keys[m] = hot[rng.integers(0, len(hot), int(m.sum()))]
    else:
        keys = rng.integers(1, max(2, n // 4), n).astype(np.uint64)
    states = np.zeros(n, np.uint8)
    if chunk > 2:
        states[:] = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.92, 0.04, 0.04])
        ends = np.arange(chunk - 1, n, chunk)
        states[ends[rng.random(len(ends)) < 0.2]] = rng.choice(np.array([1, 2], np.uint8))
    else:
        states[-3:] = [1, 0, 2][-min(3, n):]
    ids = rng.permutation(8 * n + 64)
    uniq = np.unique(keys)
    sk = uniq[rng.random(len(uniq)) < rng.uniform(0, 0.4)]
    seeds = []
    if len(sk):
        extra = sk[rng.integers(0, len(sk), len(sk) // 3)] if len(sk) > 2 else sk[:0]
        allk = np.concatenate([sk, extra])
        seeds = list(zip((int(x) for x in allk), (int(x) for x in ids[:len(allk)])))
    pre = np.full(n, NONE, np.uint32)
    own = rng.random(n) < rng.uniform(0, 0.6)
    pre[own] = ids[len(seeds):len(seeds) + int(own.sum())].astype(np.uint32)
    return keys, states, chunk, seeds, pre


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--seed", type=int, default=5)
    a = ap.parse_args()
    import torch
    from spacedrive_amd import CasEngine
    from tests.golden.make_golden import closed_form, cursor_walk, replay_identifier_job
    eng = CasEngine(0)
    rng = np.random.default_rng(a.seed)
    t0 = time.time()
    it = small = large = 0
    rows_total = 0
    while time.time() - t0 < a.seconds:
        big = it % 3 == 2
        n = int(rng.integers(20_000, 4_000_000)) if big else int(rng.integers(1, 2_500))
        keys, states, chunk, seeds, pre = draw_job(rng, n)
        sk = np.array([k for k, _ in seeds], np.uint64)
        so = np.array([o for _, o in seeds], np.uint32)
        existing = (torch.from_numpy(sk.view(np.int64)).cuda(), torch.from_numpy(so.view(np.int32)).cuda()) if len(seeds) else None
        step, obj, act, counts = eng.identifier_links(
            torch.from_numpy(keys.view(np.int64)).cuda(), torch.from_numpy(states).cuda(), chunk,
            existing=existing, pre_objects=torch.from_numpy(pre.view(np.int32)).cuda())
        gstep = step.cpu().numpy().view(np.uint32).astype(np.int64)
        gobj = obj.cpu().numpy().view(np.uint32).astype(np.int64)
        gact = act.cpu().numpy().astype(np.int64)
        if not big:
            pl = [None if int(p) == NONE else int(p) for p in pre]
            ws, wo, wa, wc = replay_identifier_job([int(k) for k in keys], [int(s) for s in states],
                                                   chunk, existing=seeds, pre_objects=pl)
            ok = ([tuple(c) for c in counts.tolist()] == wc and (gstep == np.array(ws)).all()
                  and (gobj == np.array(wo)).all() and (gact == np.array(wa)).all())
            hs, ho, ha, hc = eng.identifier_links_host(keys, states, chunk,
                                                       existing=(sk, so) if len(seeds) else None,
                                                       pre_objects=pre)
            ok = ok and (ho.astype(np.int64) == np.array(wo)).all() and (ha == np.array(wa)).all()
            small += 1
        else:
            wstep, starts, reached = cursor_walk(states, n, chunk)
            wo, wa = closed_form(keys, states, pre, seeds, wstep, starts)
            ok = bool((gstep == wstep).all() and (gobj == wo).all() and (gact == wa).all())
            large += 1
        rows_total += n
        print(json.dumps({"it": it, "n": n, "chunk": chunk, "seeds": len(seeds),
                          "owning": int((pre != NONE).sum()), "ok": bool(ok)}), flush=True)
        if not ok:
            print(json.dumps({"FAIL": it, "seed": a.seed}), flush=True)
            sys.exit(1)
        it += 1
    print(json.dumps({"summary": {"jobs": it, "small_vs_replay": small, "large_vs_closed_form": large,
                                  "rows": rows_total, "seconds": round(time.time() - t0, 1),
                                  "failures": 0}}), flush=True)


if __name__ == "__main__":
    main()
