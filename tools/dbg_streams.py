"""Debug: test_hash_regions_streams_and_ungrouped step by step on a fresh context, printing
the async Object count (sd_cas_copy_objects_dev) after every phase."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from spacedrive_amd import CasEngine  # noqa: E402

eng = CasEngine(0)
if len(sys.argv) > 1 and sys.argv[1] == "warm":
    k = torch.randint(-2**63, 2**63 - 1, (9_000_000,), dtype=torch.int64, device="cuda")
    r = torch.empty(9_000_000, dtype=torch.int32, device="cuda")
    eng.group(k, r)
    del k, r
q = eng.batch_quantum
n = q
s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
data = []
for j in range(5):
    c = torch.empty((n, 57344), dtype=torch.uint8, device="cuda")
    z = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_sampled(300 + j, j * n, n, c, z, 57344, dup_permille=300)
    data.append((c, z))
torch.cuda.synchronize()
ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
keys = [torch.empty(n, dtype=torch.int64, device="cuda") for _ in range(5)]
reps = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(5)]
obj = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(5)]


def cobj(tag, stream):
    t = torch.zeros(1, dtype=torch.int64, device="cuda")
    eng._check(eng.L.sd_cas_copy_objects_dev(eng.h, t.data_ptr(), stream), "copy")
    torch.cuda.synchronize()
    print(tag, int(t.item()), flush=True)


plan = [(s1, True), (s2, False), (s1, True), (s2, True), (s1, True)]
for j, ((c, z), (st, grp)) in enumerate(zip(data, plan)):
    eng.hash_regions_sampled(c, z, keys[j], reps[j], ovf, stream=st.cuda_stream)
    if grp:
        eng.group_regions(n, reps[j], stream=s3.cuda_stream, want_objects=False)
        eng._check(eng.L.sd_cas_copy_objects_dev(eng.h, obj[j].data_ptr(), s3.cuda_stream), "copy")
torch.cuda.synchronize()
print("obj", [int(o.item()) for o in obj])
cobj("after loop (s3)", s3.cuda_stream)
for j in (0, 2, 3, 4):
    rep = torch.empty(n, dtype=torch.int32, device="cuda")
    print("group", j, eng.group(keys[j], rep), torch.equal(rep, reps[j]))
cobj("after groups (s3)", s3.cuda_stream)
cobj("after groups (null)", 0)
eng.hash_regions_sampled(data[0][0], data[0][1], keys[0], reps[0], ovf, stream=s1.cuda_stream)
torch.cuda.synchronize()
cobj("after refill 1 (s3)", s3.cuda_stream)
eng.hash_regions_sampled(data[1][0], data[1][1], keys[1], reps[1], ovf, stream=s2.cuda_stream)
torch.cuda.synchronize()
cobj("after refill 2 (s3)", s3.cuda_stream)
