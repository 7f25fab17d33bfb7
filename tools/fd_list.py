# fd_list.py (round 6): the descriptors a process holds before and after HIP init + a context
# and one gather (what the pool threads private tables start from).
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
def show(tag):
    out = []
    for fd in sorted(os.listdir("/proc/self/fd"), key=int):
        try:
            out.append(f"{fd} -> {os.readlink('/proc/self/fd/' + fd)}")
        except OSError:
            pass
    print(tag, len(out)); print("\n".join(out)); sys.stdout.flush()
show("before_hip")
import torch
torch.zeros(1, device="cuda")
from spacedrive_amd import CasEngine
import numpy as np
e = CasEngine(0)
p = "/tmp/fdlist_probe.bin"
open(p, "wb").write(os.urandom(300000))
print(e.file_checksums([p] * 40)[1].any())
show("after_hip_and_ctx")
