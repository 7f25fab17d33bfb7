"""Config-1 drop-in timing for A/B (no CPU oracle): sd_cas_generate_cas_ids_from_paths over a
file list made by tools/gpu_r3_ab_c1.sh ("path size" lines), 1 warm call + 5 timed calls,
keys digest printed (variants must agree).  Library from SD_HIP_CAS_LIB."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spacedrive_amd import CasEngine  # noqa: E402

paths, sizes = [], []
for line in open(sys.argv[1]):
    p, s = line.split()
    paths.append(p)
    sizes.append(int(s))
eng = CasEngine(0)
keys, st = eng.generate_cas_keys_from_paths(paths, sizes)
assert not st.any()
ts = []
for _ in range(5):
    t = time.perf_counter()
    k2, _ = eng.generate_cas_keys_from_paths(paths, sizes)
    ts.append(time.perf_counter() - t)
    assert (k2 == keys).all()
print(json.dumps({"lib": os.path.basename(os.environ.get("SD_HIP_CAS_LIB", "current")),
                  "ms": [round(x * 1e3, 2) for x in ts], "median_ms": float(np.median(ts)) * 1e3,
                  "files_per_s": len(paths) / float(np.median(ts)),
                  "digest": f"{int((keys * np.uint64(0x9E3779B97F4A7C15)).sum()):016x}"}), flush=True)
