"""A/B of the fused hash + group chain (sd_cas_hash_group_sampled_dev: K1G + one bucket-table
launch) against K1 alone and against K1 followed by the standalone grouping chain, on one
resident sampled batch (30 % duplicates), interleaved; every fused result checked against
the standalone grouping (rep and Object count) and the keys against K1's.  HIP events on the
context's stream.  Prints one JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spacedrive_amd import CasEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--files", type=int, default=1_310_720)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--group-reps", type=int, default=20)
ap.add_argument("--hot", type=int, nargs="*", default=[],
                help="copies of hot files (one file each) spread over the batch: the fused "
                     "chain's region-overflow path (regrouped on the device per region)")
a = ap.parse_args()
eng = CasEngine(0)
dev = torch.device("cuda", 0)
F = a.files
content = torch.empty((F, 57344), dtype=torch.uint8, device=dev)
sizes = torch.empty(F, dtype=torch.int64, device=dev)
keys = torch.empty(F, dtype=torch.int64, device=dev)
keys2 = torch.empty(F, dtype=torch.int64, device=dev)
rep = torch.empty(F, dtype=torch.int32, device=dev)
rep2 = torch.empty(F, dtype=torch.int32, device=dev)
ovf = torch.zeros(1, dtype=torch.int32, device=dev)
eng.synth_sampled(7, 0, F, content, sizes, 57344, dup_permille=300)
_g = np.random.default_rng(5)
for h, copies in enumerate(a.hot):
    idx = torch.from_numpy(_g.choice(np.arange(len(a.hot), F), copies, replace=False)).to(dev)
    content[idx] = content[h].clone()
    sizes[idx] = sizes[h].clone()
s = torch.cuda.Stream()


def timed(fn, reps=1):
    a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        a_.record(s)
        for _ in range(reps):
            fn()
        b_.record(s)
    b_.synchronize()
    return a_.elapsed_time(b_) / reps


cs = lambda: s.cuda_stream  # noqa: E731
k1 = lambda: eng.hash_sampled(content, sizes, keys, stream=cs())  # noqa: E731
grp = lambda: eng.group(keys, rep, stream=cs(), want_objects=False)  # noqa: E731
fused = lambda: eng.hash_group_sampled(content, sizes, keys2, rep2, ovf, stream=cs(), want_objects=False)  # noqa: E731
regions = lambda: eng.hash_regions_sampled(content, sizes, keys2, rep2, ovf, stream=cs())  # noqa: E731
tables = lambda: eng.group_regions(F, rep2, stream=cs(), want_objects=False)  # noqa: E731
k1(); grp(); fused()  # warm
torch.cuda.synchronize()
res = {"k1": [], "k1_then_group": [], "fused": [], "group_alone": [], "tables_alone": []}
for _ in range(a.reps):
    res["k1"].append(timed(k1))
    res["k1_then_group"].append(timed(lambda: (k1(), grp())))
    res["fused"].append(timed(fused))
    res["group_alone"].append(timed(grp, a.group_reps))
    regions()
    res["tables_alone"].append(timed(tables))
torch.cuda.synchronize()
ovf.zero_()
obj_std = eng.group(keys, rep)
obj_fused = eng.hash_group_sampled(content, sizes, keys2, rep2, ovf)
torch.cuda.synchronize()
parity = bool(torch.equal(keys, keys2) and torch.equal(rep, rep2) and obj_std == obj_fused)
med = {k: float(np.median(v)) for k, v in res.items()}
print(json.dumps({"files": F, "hot_copies": a.hot, "median_ms": med, "all_ms": res, "objects": obj_std,
                  "overflow": int(ovf.item()), "parity_fused_vs_standalone": parity,
                  "fused_minus_k1_ms": med["fused"] - med["k1"],
                  "k1_then_group_minus_k1_ms": med["k1_then_group"] - med["k1"]}), flush=True)
