#!/bin/bash
# Round 3: host-side config-1 gather scaling on the GPU box (tools/ubench_gather.c): the
# product gather's syscall pattern over BASELINE config 1's 10k tmpfs files at 1-16
# threads, with pread and with io_uring.  CPU only.  Usage: <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3_gather}
mkdir -p $OUT
cd $R
gcc -O2 -pthread -o $OUT/ubench_gather tools/ubench_gather.c || exit 1
D=/dev/shm/sdcas_gather_$$
python3 - "$D" > $OUT/list.txt <<'PY'
import math, os, sys
import numpy as np
d = sys.argv[1]; os.makedirs(d, exist_ok=True)
rng = np.random.default_rng(1)
sizes = np.exp(rng.uniform(math.log(1024), math.log(10 * 1024 * 1024), 10000)).astype(np.int64)
for i, s in enumerate(sizes):
    p = f"{d}/f{i:05d}"
    with open(p, "wb") as fh:
        fh.write(rng.integers(0, 256, int(s), dtype=np.uint8).tobytes())
    print(p, int(s))
PY
for T in 1 4 8 16 32; do timeout -k 5 120 $OUT/ubench_gather $OUT/list.txt $T | tail -2; done > $OUT/gather.log 2>&1
for T in 1 16; do timeout -k 5 120 $OUT/ubench_gather $OUT/list.txt $T uring | tail -2; done >> $OUT/gather.log 2>&1
nproc >> $OUT/gather.log; grep -m1 "model name" /proc/cpuinfo >> $OUT/gather.log
rm -rf $D
cat $OUT/gather.log
