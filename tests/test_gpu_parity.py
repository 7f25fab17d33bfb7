"""GPU parity tests (MI355X): the HIP path through the C ABI vs the oracle, bit-exact.

Covers every hot-path row of SURVEY.md §8a that the build implements: K1 sampled cas,
K2 whole-file cas (ragged lengths, the inclusive 100 KiB edge, the 8-byte tail chunk),
the host drop-ins (buffers and paths, with per-file I/O errors), grouping (canonical and
the chunk-of-100 replay), the radix sort, the validator checksum (device buffer and
streamed file), and — at BASELINE sizes — size-independent properties.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle.pyoracle import MINIMUM_FILE_SIZE, SAMPLED_CONTENT_LEN, np_content, py_sample_plan
from tests.golden.make_golden import canonical, gather_virtual, replay_identifier, replay_identifier_job

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def dev64(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host64(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)


def sampled_batch(rng, n, stride=SAMPLED_CONTENT_LEN):
    content = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    sizes = rng.integers(MINIMUM_FILE_SIZE + 1, 2 ** 40, n, dtype=np.uint64)
    return content, sizes


# Each device-hash test runs every kernel shape: threshold 0 forces the lane-per-file
# kernels (K1/K2) at every n, a huge threshold forces the chunk-parallel K1L — with a wave
# per file (split huge) or four files per wave with DPP cross-lane merges (split 0).
PATHS = {"lane": (0, None), "chunkpar": (1 << 40, 1 << 40), "chunkpar16": (1 << 40, 0)}


@pytest.fixture(params=list(PATHS))
def path_eng(eng, request):
    thr, split = PATHS[request.param]
    eng.set_latency_threshold(thr, thr)
    eng.set_chunkpar_split(split, split)
    yield eng
    eng.set_latency_threshold()
    eng.set_chunkpar_split()


def test_sampled_kernel_vs_oracle(path_eng, oracle):
    eng = path_eng
    rng = np.random.default_rng(1)
    for n, stride in [(1, SAMPLED_CONTENT_LEN), (63, SAMPLED_CONTENT_LEN), (1000, SAMPLED_CONTENT_LEN),
                      (257, SAMPLED_CONTENT_LEN + 48)]:
        content, sizes = sampled_batch(rng, n, stride)
        want = oracle.fast_cas_keys_strided(content.reshape(-1), stride, SAMPLED_CONTENT_LEN, sizes, 8)
        keys = torch.zeros(n, dtype=torch.int64, device="cuda")
        eng.hash_sampled(torch.from_numpy(content).cuda(), dev64(sizes), keys, stride=stride)
        assert (host64(keys) == want).all(), (n, stride)


def test_sampled_golden(path_eng, golden):
    eng = path_eng
    g = golden["cas"]
    files = [f for f in g["files"] if f["size"] > MINIMUM_FILE_SIZE]
    content = np.stack([np.frombuffer(gather_virtual(g["seed"], f["file"], f["size"]), np.uint8)
                        for f in files])
    sizes = np.array([f["size"] for f in files], dtype=np.uint64)
    keys = torch.zeros(len(files), dtype=torch.int64, device="cuda")
    eng.hash_sampled(torch.from_numpy(content).cuda(), dev64(sizes), keys)
    got = [f"{k:016x}" for k in host64(keys)]
    assert got == [f["cas_id"] for f in files]


def packed_arena(contents):
    offs, o = [], 0
    for c in contents:
        offs.append(o)
        o += (len(c) + 15) // 16 * 16
    arena = np.zeros(o + 128, dtype=np.uint8)  # readable to every content's 128-B round-up
    for c, off in zip(contents, offs):
        arena[off:off + len(c)] = np.frombuffer(c, np.uint8)
    return arena, np.array(offs, dtype=np.uint64)


EDGE_LENS = (list(range(0, 130)) + [1015, 1016, 1017, 1023, 1024, 1025, 2040, 2041, 2047, 2048,
             4088, 4096, 16376, 32760, 65528, 102399, 102400, 57344, 104000, 104 * 1024 - 8])


def test_packed_kernel_edges_vs_oracle(path_eng, oracle):
    eng = path_eng
    rng = np.random.default_rng(2)
    lens = EDGE_LENS + [int(x) for x in rng.integers(0, 102401, 1500)]
    contents = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
    # neighbour garbage must not leak into a message: fill the padding with 0xFF
    arena, offs = packed_arena(contents)
    for c, off in zip(contents, offs):
        pad = (len(c) + 15) // 16 * 16 - len(c)
        arena[off + len(c): off + len(c) + pad] = 0xFF
    sizes = np.array([L if L <= MINIMUM_FILE_SIZE else L * 3 + 200_000 for L in lens], dtype=np.uint64)
    want = oracle.cas_keys(arena, offs, np.array(lens, dtype=np.uint64), sizes)
    keys = torch.zeros(len(lens), dtype=torch.int64, device="cuda")
    eng.hash_packed(torch.from_numpy(arena).cuda(), dev64(offs),
                    torch.tensor(lens, dtype=torch.int32, device="cuda"), dev64(sizes), keys)
    got = host64(keys)
    bad = [(lens[i], f"{got[i]:016x}", f"{want[i]:016x}") for i in range(len(lens)) if got[i] != want[i]]
    assert not bad, bad[:10]


def test_host_generate_cas_ids_mixed(path_eng, oracle, golden):
    eng = path_eng
    g = golden["cas"]
    items = [(gather_virtual(g["seed"], f["file"], f["size"]), f["size"]) for f in g["files"]]
    assert eng.generate_cas_ids(items) == [f["cas_id"] for f in g["files"]]
    rng = np.random.default_rng(3)
    items = []
    for i in range(300):
        if rng.random() < 0.5:
            s = int(rng.integers(MINIMUM_FILE_SIZE + 1, 2 ** 33))
            items.append((rng.integers(0, 256, SAMPLED_CONTENT_LEN, dtype=np.uint8).tobytes(), s))
        else:
            s = int(rng.integers(0, MINIMUM_FILE_SIZE + 1))
            items.append((rng.integers(0, 256, s, dtype=np.uint8).tobytes(), s))
    assert eng.generate_cas_ids(items) == [oracle.cas_id(b, s) for b, s in items]
    with pytest.raises(Exception):
        eng.generate_cas_ids([(b"x" * 100, 10 ** 7)])  # sampled size needs 57,344 bytes


def test_generate_from_paths_and_errors(eng, oracle, tmp_path):
    import spacedrive_amd as sd
    rng = np.random.default_rng(4)
    paths, sizes, imgs = [], [], []
    for i, size in enumerate([1, 100, 1024, 102400, 102401, 250_000, 3_000_001]):
        img = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        p = tmp_path / f"f{i}"
        p.write_bytes(img)
        paths.append(str(p)); sizes.append(size); imgs.append(img)
    paths.append(str(tmp_path / "missing")); sizes.append(5000)
    short = tmp_path / "short"
    short.write_bytes(b"z" * 120_000)
    paths.append(str(short)); sizes.append(10 ** 7)  # stale metadata: read_exact -> EOF
    # stale metadata on the whole-file path: cas.rs:29 hashes le64(size) || the file as it
    # is now (shrunk; grown within, and far beyond, the whole-file message limit)
    for j, (actual, size) in enumerate([(3000, 5000), (90_000, 1000), (300_000, 50)]):
        p = tmp_path / f"stale{j}"
        p.write_bytes(rng.integers(0, 256, actual, dtype=np.uint8).tobytes())
        paths.append(str(p)); sizes.append(size)
    keys, errs = eng.generate_cas_keys_from_paths(paths, sizes)
    for i in list(range(7)) + [9, 10, 11]:
        assert errs[i] == 0, i
        assert f"{keys[i]:016x}" == oracle.generate_cas_id(paths[i], sizes[i]), i
    assert errs[7] == -2  # ENOENT
    assert errs[8] == -5  # EIO (UnexpectedEof)
    # the single-file drop-in raises like io::Error
    assert sd.generate_cas_id(paths[5], sizes[5]) == oracle.generate_cas_id(paths[5], sizes[5])
    with pytest.raises(OSError):
        sd.generate_cas_id(paths[7], 5000)


def test_from_paths_stale_sampled_footer(eng, oracle, tmp_path):
    """Sampled files whose length changed after fs::metadata: the footer comes from the
    file's actual end (cas.rs:54-55 SeekFrom::End), samples from `size`; grown files and
    shrunk-but-readable files get the reference's cas_id, files shrunk below a sample fail
    with EIO — each vs the literal read/seek execution and the C oracle."""
    from oracle.pyoracle import UnexpectedEof, py_generate_cas_id_file
    from tests.test_oracle import stale_files
    files = stale_files(tmp_path)
    keys, errs = eng.generate_cas_keys_from_paths([p for p, _ in files], [s for _, s in files])
    for (path, size), k, e in zip(files, keys, errs):
        try:
            want = py_generate_cas_id_file(path, size)
        except UnexpectedEof:
            want = None
        if want is None:
            assert e == -5 and k == 0, (path, size)
        else:
            assert e == 0 and f"{k:016x}" == want == oracle.generate_cas_id(path, size), (path, size)


def test_from_paths_windowed_pipeline(eng, oracle, tmp_path):
    """> 2 gather windows (2,048 files each): slots reused, errors in several windows."""
    rng = np.random.default_rng(14)
    n = 5000
    sizes = [int(s) for s in np.exp(rng.uniform(0, np.log(400_000), n)).astype(np.int64)]
    paths = []
    for i, s in enumerate(sizes):
        p = tmp_path / f"g{i}"
        if i % 997 != 13:  # a missing file in each window
            p.write_bytes(rng.integers(0, 256, s, dtype=np.uint8).tobytes())
        paths.append(str(p))
    keys, errs = eng.generate_cas_keys_from_paths(paths, sizes)
    for i in range(n):
        if i % 997 == 13:
            assert errs[i] == -2 and keys[i] == 0, i
        else:
            assert errs[i] == 0, i
    check = [i for i in range(n) if i % 997 != 13][::7]
    bad = [i for i in check if f"{keys[i]:016x}" != oracle.generate_cas_id(paths[i], sizes[i])]
    assert not bad, bad[:5]


@pytest.mark.parametrize("kind", ["sampled", "whole", "mixed"])
def test_from_paths_job_step_shapes(eng, oracle, tmp_path, kind):
    """The reference's 100-file job step (mod.rs:34) through the single-window path whose H2D
    streams behind the gather: all-sampled (no packed area but its pad), all-whole, mixed,
    with a missing file, and 16/17/99/100/101-file batches around the streaming threshold."""
    rng = np.random.default_rng({"sampled": 31, "whole": 32, "mixed": 33}[kind])
    lo, hi = {"sampled": (150_000, 3_000_000), "whole": (1, 100_000), "mixed": (1, 3_000_000)}[kind]
    paths, sizes = [], []
    for i in range(101):
        s = int(np.exp(rng.uniform(np.log(lo), np.log(hi))))
        p = tmp_path / f"{kind}{i:03d}"
        if i != 57:
            p.write_bytes(rng.integers(0, 256, s, dtype=np.uint8).tobytes())
        paths.append(str(p))
        sizes.append(s)
    for m in (15, 16, 17, 99, 100, 101):
        keys, errs = eng.generate_cas_keys_from_paths(paths[:m], sizes[:m])
        for i in range(m):
            if i == 57:
                assert errs[i] == -2 and keys[i] == 0
            else:
                assert errs[i] == 0 and f"{keys[i]:016x}" == oracle.generate_cas_id(paths[i], sizes[i]), (m, i)


@pytest.mark.parametrize("shape", ["default", "seg16", "lane"])
def test_from_paths_streamed_mixed_edge_rows(eng, oracle, tmp_path, shape):
    """The streamed single-window path (>= 16 files, whole files read, sent and hashed first,
    the sampled pieces after them) with every kind of row the gather decides: stale whole
    files (shrunk, grown within and beyond the whole-file limit: re-read after the window),
    a stale sampled file (UnexpectedEof -> EIO), a missing file, a directory (EISDIR), a
    caller size of 0 (NO_CAS, nothing read) — under the default kernel shapes, the sorted
    four-files-per-wave K1L, and the lane-per-file kernels."""
    import errno

    import spacedrive_amd as sd
    rng = np.random.default_rng(41)
    paths, sizes = [], []
    for i in range(48):
        s = int(np.exp(rng.uniform(np.log(10), np.log(2_500_000))))
        p = tmp_path / f"e{i:02d}"
        p.write_bytes(rng.integers(0, 256, s, dtype=np.uint8).tobytes())
        paths.append(str(p))
        sizes.append(s)
    for j, (actual, size) in enumerate([(3000, 5000), (90_000, 1000), (300_000, 50)]):
        p = tmp_path / f"stale{j}"
        p.write_bytes(rng.integers(0, 256, actual, dtype=np.uint8).tobytes())
        paths.insert(5 + 7 * j, str(p))
        sizes.insert(5 + 7 * j, size)
    short = tmp_path / "short"
    short.write_bytes(b"z" * 120_000)
    paths.insert(30, str(short)); sizes.insert(30, 10 ** 7)
    paths.insert(33, str(tmp_path / "missing")); sizes.insert(33, 5000)
    os.mkdir(str(tmp_path / "adir"))
    paths.insert(40, str(tmp_path / "adir")); sizes.insert(40, 4096)
    sizes[44] = 0
    if shape == "seg16":
        eng.set_chunkpar_split(0, 0)
    elif shape == "lane":
        eng.set_latency_threshold(0, 0)
    try:
        keys, status = eng.generate_cas_keys_from_paths(paths, sizes)
    finally:
        eng.set_latency_threshold()
        eng.set_chunkpar_split()
    for i, (p, s) in enumerate(zip(paths, sizes)):
        if i == 30:
            assert status[i] == -errno.EIO and keys[i] == 0
        elif i == 33:
            assert status[i] == -errno.ENOENT and keys[i] == 0
        elif i == 40:
            assert status[i] in (-errno.EISDIR,) and keys[i] == 0
        elif i == 44:
            assert status[i] == sd.cas.STATUS_NO_CAS and keys[i] == 0
        else:
            assert status[i] == 0 and f"{keys[i]:016x}" == oracle.generate_cas_id(p, s), (shape, i, s)


def test_from_paths_file_metadata_rules(eng, oracle, tmp_path):
    """FileMetadata::new's rules behind the ABI (file_identifier/mod.rs:55-95): with the
    metadata taken by the library (sizes NULL) a file emptied after it was indexed gets no
    cas_id (SD_CAS_STATUS_NO_CAS, key 0), a directory is refused with EISDIR (the reference
    asserts, :67-70), a missing path is ENOENT, a symlink is followed (fs::metadata); with
    caller sizes a 0 is NO_CAS without any read.  The rows then go through the link emission
    vs the literal job replay, the NO_CAS row at a chunk end included."""
    import errno

    import spacedrive_amd as sd
    from oracle.pyoracle import py_generate_cas_id_file
    rng = np.random.default_rng(31)
    paths, indexed = [], []
    for i in range(14):
        p = tmp_path / f"m{i:02d}"
        size = [700, 102400, 102401, 333_333][i % 4]
        p.write_bytes(rng.integers(0, 256, size, dtype=np.uint8).tobytes())
        paths.append(str(p))
        indexed.append(size)
    # row 5 (the last row of the second chunk of 3): emptied after indexing
    with open(paths[5], "wb"):
        pass
    os.symlink(paths[2], str(tmp_path / "link"))
    paths[8] = str(tmp_path / "link")
    os.mkdir(str(tmp_path / "adir"))
    paths[10] = str(tmp_path / "adir")
    paths[12] = str(tmp_path / "gone")
    keys, status = eng.generate_cas_keys_from_paths(paths, None)
    states, want_keys = [], []
    for i, p in enumerate(paths):
        if i == 5:
            assert status[i] == sd.cas.STATUS_NO_CAS and keys[i] == 0
            states.append(1); want_keys.append(0)
        elif i == 10:
            assert status[i] == -errno.EISDIR and keys[i] == 0
            states.append(2); want_keys.append(0)
        elif i == 12:
            assert status[i] == -errno.ENOENT and keys[i] == 0
            states.append(2); want_keys.append(0)
        else:
            size = os.stat(p).st_size
            want = py_generate_cas_id_file(p, size)
            assert status[i] == 0 and f"{keys[i]:016x}" == want == oracle.generate_cas_id(p, size), i
            states.append(0); want_keys.append(int(want, 16))
    # caller-given metadata: a length of 0 is NO_CAS (not read), a directory still EISDIR
    k2, s2 = eng.generate_cas_keys_from_paths([paths[5], paths[10], paths[0]], [0, 4096, 700])
    assert list(s2) == [sd.cas.STATUS_NO_CAS, -errno.EISDIR, 0] and k2[0] == 0 and k2[2] == keys[0]
    # ... also when the caller's metadata puts the directory on the sampled path (its first
    # read fails: no fstat ahead of a sampled file's reads)
    k3, s3 = eng.generate_cas_keys_from_paths([paths[10]] * 20, [10_000_000] * 20)
    assert (s3 == -errno.EISDIR).all() and not k3.any()
    # the job over these rows: decisions and per-step batches vs the literal replay
    for chunk in (3, 100):
        res = sd.identifier_job_step(paths, chunk=chunk, eng=eng)
        step, obj, act, counts, creates = replay_identifier_job(want_keys, states, chunk, with_creates=True)
        assert res.errors == {10: errno.EISDIR, 12: errno.ENOENT}
        assert [(b.total_created, b.total_linked) for b in res.steps] == counts
        assert [b.creates for b in res.steps] == creates
        assert {i: o for i, (o, a) in enumerate(zip(obj, act)) if a in (0, 1)} == res.object_of
        assert res.metadata[5].cas_id is None
    assert 5 in res.steps[0].creates  # chunk 100: one step
    res3 = sd.identifier_job_step(paths, chunk=3, eng=eng)
    assert 5 in res3.steps[1].creates and 5 in res3.steps[2].creates  # re-queried NO_CAS row


def test_sort_pairs_vs_numpy(eng):
    """Tile (4,096 keys) and count-block (4 tiles) boundaries included: a block's last tile
    partial, a lone tile in the last block, several scan batches per block range."""
    rng = np.random.default_rng(5)
    for n in [1, 255, 4096, 4097, 16_383, 16_384, 16_385, 20_481, 100_003, 1_000_003]:
        k = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
        k[: n // 3] = k[n // 2] if n > 2 else k[0]  # ties: stability matters
        ko = torch.empty(n, dtype=torch.int64, device="cuda")
        vo = torch.empty(n, dtype=torch.int32, device="cuda")
        eng.sort_pairs(dev64(k), None, ko, vo)
        order = np.argsort(k, kind="stable")
        assert (host64(ko) == k[order]).all()
        assert (vo.cpu().numpy() == order).all()
        # top-byte partition pass (the multi-GPU split) is stable on the top 8 bits
        eng.sort_pairs(dev64(k), None, ko, vo, 56, 64)
        order = np.argsort(k >> np.uint64(56), kind="stable")
        assert (vo.cpu().numpy() == order).all()
        # caller values and a bit range whose last digit is narrower than 8 bits
        v = rng.permutation(n).astype(np.int32)
        eng.sort_pairs(dev64(k), torch.from_numpy(v).cuda(), ko, vo, 3, 23)
        order = np.argsort((k >> np.uint64(3)) & np.uint64((1 << 20) - 1), kind="stable")
        assert (vo.cpu().numpy() == v[order]).all() and (host64(ko) == k[order]).all()


def test_sort_pairs_repeated_large(eng):
    """The downsweep's per-round wave counts race if a wave runs a round ahead (a lost count
    misplaces keys in ~1 of 10^7): repeat 12.5 M-key sorts — one rank's share at config 4 —
    and compare every run with numpy's stable order."""
    rng = np.random.default_rng(55)
    n = 12_500_000
    k = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
    k[n // 2:] = k[: n - n // 2]  # every key twice: stability matters
    order = np.argsort(k, kind="stable").astype(np.int32)
    dk = dev64(k)
    ko = torch.empty(n, dtype=torch.int64, device="cuda")
    vo = torch.empty(n, dtype=torch.int32, device="cuda")
    want = torch.from_numpy(order).cuda()
    for it in range(12):
        eng.sort_pairs(dk, None, ko, vo)
        assert bool((vo == want).all()), it


def test_group_vs_oracle(eng, oracle, golden):
    for name, lay in golden["grouping"]["layouts"].items():
        keys = np.array([int(k, 16) for k in lay["keys"]], dtype=np.uint64)
        rep = torch.empty(len(keys), dtype=torch.int32, device="cuda")
        objects = eng.group(dev64(keys), rep)
        assert rep.cpu().tolist() == lay["rep"] and objects == lay["objects"], name
        rc = torch.empty_like(rep)
        c, ln = eng.group_chunked(rep, rc, 100)
        assert rc.cpu().tolist() == lay["rep_chunked"] and (c, ln) == (lay["created"], lay["linked"]), name
    rng = np.random.default_rng(6)
    for n, pool in [(1, 1), (5000, 5000), (300_001, 50_000), (50_000, 1), (1 << 20, 700_000)]:
        base = rng.integers(0, 2 ** 64, pool, dtype=np.uint64)
        keys = base[rng.integers(0, pool, n)]
        rep = torch.empty(n, dtype=torch.int32, device="cuda")
        objects = eng.group(dev64(keys), rep)
        orep, oobj = oracle.group_canonical(keys)
        assert objects == oobj
        assert (rep.cpu().numpy().astype(np.uint32) == orep).all()
        rc = torch.empty_like(rep)
        c, ln = eng.group_chunked(rep, rc, 100)
        crep, cc, cl = oracle.group_chunked(keys, 100)
        assert (c, ln) == (cc, cl) and (rc.cpu().numpy().astype(np.uint32) == crep).all()


MASK64 = (1 << 64) - 1


def unmix64(m: int) -> int:
    """Inverse of the splitmix64 finalizer the hash grouping buckets by (group_hash.hip)."""
    def unxorshift(z, s):
        x = z
        for _ in range(64 // s + 1):
            x = z ^ (x >> s)
        return x & MASK64
    m = unxorshift(m, 31)
    m = (m * pow(0x94D049BB133111EB, -1, 1 << 64)) & MASK64
    m = unxorshift(m, 27)
    m = (m * pow(0xBF58476D1CE4E5B9, -1, 1 << 64)) & MASK64
    return unxorshift(m, 30)


def test_group_hash_adversarial_keys(eng, oracle):
    """K4h/K5h on key sets that are not uniform: small integers, one key repeated,
    8,000 distinct keys crafted (inverse mix) into ONE bucket so its LDS table overflows
    and the global-memory table takes over, and keys ordered by bucket (maximally unequal
    per-replica sub-runs in the scatter) — every case vs the oracle's canonical grouping."""
    rng = np.random.default_rng(40)
    crafted = np.array([unmix64(int(x) >> 3) for x in rng.integers(0, 2 ** 63, 8000, dtype=np.uint64)],
                       dtype=np.uint64)  # mix64(key) has top 3 bits 0: all in bucket 0 of 8
    cases = {
        "small ints": rng.integers(0, 3000, 9000, dtype=np.uint64),
        "iota": np.arange(70_000, dtype=np.uint64),
        "one key": np.full(100_000, 0xDEADBEEF, dtype=np.uint64),
        "zero and max": rng.choice(np.array([0, 2 ** 64 - 1], dtype=np.uint64), 5000),
        "crafted overflow": crafted[rng.integers(0, len(crafted), 12_000)],
        "crafted distinct": crafted,
    }
    # two-level partition (> 786K keys) with one fine bucket overflowing: 10K distinct keys
    # whose mixed top 14 bits are 0, among 1M uniform keys
    deep = np.array([unmix64(int(x) >> 14) for x in rng.integers(0, 2 ** 63, 10_000, dtype=np.uint64)],
                    dtype=np.uint64)
    # <= 1.44M keys: one level into 256 coarse buckets, 12,288-slot tables (sd_bucket_min_big);
    # above: the refine level and 4,096-slot tables — one overflowing bucket in each
    big = np.concatenate([rng.integers(0, 2 ** 64, 990_000, dtype=np.uint64), deep])
    cases["big-table overflow"] = big[rng.permutation(len(big))]
    big = np.concatenate([rng.integers(0, 2 ** 64, 1_600_000, dtype=np.uint64), deep])
    cases["two-level overflow"] = big[rng.permutation(len(big))]
    # keys ordered by their mixed value: every partition block's slice falls in a few
    # buckets, so the per-replica sub-runs of a bucket (the scatter's reservation ranges)
    # are as unequal as they can be — one level (1.2M) and two levels (3M), ascending and
    # descending
    from oracle.pyoracle import np_mix64
    for label, m in (("1 level", 1_200_000), ("2 levels", 3_000_000)):
        sk = rng.integers(0, 2 ** 64, m, dtype=np.uint64)
        sk[1::4] = sk[0::4][: len(sk[1::4])]
        order = np.argsort(np_mix64(sk), kind="stable")
        cases[f"bucket-sorted {label}"] = sk[order]
        cases[f"bucket-sorted desc {label}"] = sk[order[::-1]]
    for name, keys in cases.items():
        rep = torch.empty(len(keys), dtype=torch.int32, device="cuda")
        objects = eng.group(dev64(keys), rep)
        orep, oobj = oracle.group_canonical(keys)
        assert objects == oobj, name
        assert (rep.cpu().numpy().astype(np.uint32) == orep).all(), name


@pytest.mark.parametrize("method,target,n", [
    (2, 0, 300_001),          # LSD sort + run heads (the path above the hash range)
    (1, 16, 300_001),         # hash plan b1 = 8, b2 = 7 with ~18-key buckets
    (1, 16, 5_000_000),       # b1 = 9, b2 = 9: the > 200M-key plan shape
    (1, 16, 9_000_000),       # b1 = 10, b2 = 9: the deepest plan (2^19 buckets)
])
def test_group_methods_and_deep_plans(eng, oracle, method, target, n):
    """Every grouping method / partition depth gives the canonical grouping: forced LSD,
    and hash plans with a small bucket target so that the partition shapes of >200M keys
    (coarse levels of 2^9 / 2^10 buckets, 2^9-way refine) run at test sizes — for
    sd_cas_group_dev vs the oracle and sd_cas_group_min_dev (random u32 vals) vs numpy."""
    rng = np.random.default_rng(70 + n % 97)
    pool = rng.integers(0, 2 ** 64, max(1, n * 2 // 3), dtype=np.uint64)
    keys = pool[rng.integers(0, len(pool), n)]
    eng.set_group_method(method, target)
    try:
        rep = torch.empty(n, dtype=torch.int32, device="cuda")
        objects = eng.group(dev64(keys), rep)
        orep, oobj = oracle.group_canonical(keys)
        assert objects == oobj
        assert (rep.cpu().numpy().astype(np.uint32) == orep).all()
        vals = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        objects = eng.group_min(dev64(keys), torch.from_numpy(vals.view(np.int32)).cuda(), out)
        uniq, inv = np.unique(keys, return_inverse=True)
        mins = np.full(len(uniq), 0xFFFFFFFF, dtype=np.uint32)
        np.minimum.at(mins, inv, vals)
        assert objects == len(uniq)
        assert (out.cpu().numpy().view(np.uint32) == mins[inv]).all()
    finally:
        eng.set_group_method()


def test_lsd_group_runs_across_tiles(eng, oracle):
    """The LSD grouping's runs kernel (round 6: heads + rep in one pass, a run entering a tile
    found by a galloping lower bound): runs that end exactly at, one before and one after the
    4,096-key tile boundaries, runs spanning many tiles, one key everywhere, 0 and 2^64-1,
    hot keys among uniform ones — through sd_cas_group_dev (SD_CAS_GROUP_SORT: rep laid down
    by the iota sort, only duplicates stored), the public sort_pairs + group_sorted pair
    (every rep stored) and sd_cas_group_min_dev (two sorts), each vs the canonical grouping."""
    rng = np.random.default_rng(61)
    T = 4096
    counts = [T, T, 1, T - 1, 2 * T, 3, T - 2, 1, 1, 5 * T + 7, 17, T + 1, 40 * T, 2, 9]
    tiled = np.repeat(rng.integers(0, 2 ** 64, len(counts), dtype=np.uint64), counts)
    hot = np.concatenate([rng.integers(0, 2 ** 64, 300_000, dtype=np.uint64),
                          np.full(70_000, 0x1234, dtype=np.uint64),
                          np.full(9_000, 2 ** 64 - 1, dtype=np.uint64), np.zeros(5000, dtype=np.uint64)])
    pool = rng.integers(0, 2 ** 64, 700, dtype=np.uint64)
    cases = {
        "tile-aligned runs": tiled[rng.permutation(len(tiled))],
        "tile-aligned runs, input sorted": np.sort(tiled),
        "one key": np.full(3 * T * 25 + 5, 0xABCDEF, dtype=np.uint64),
        "hot keys": hot[rng.permutation(len(hot))],
        "few keys, long runs": pool[rng.integers(0, len(pool), 1_000_003)],
        "30% dups at a tile multiple": None,
    }
    u = rng.integers(0, 2 ** 64, 7 * T * 10 // 10, dtype=np.uint64)
    cases["30% dups at a tile multiple"] = np.concatenate([u, u[rng.integers(0, len(u), 10 * T - len(u))]])
    for name, keys in cases.items():
        n = len(keys)
        orep, oobj = oracle.group_canonical(keys)
        eng.set_group_method(eng.GROUP_SORT)
        try:
            rep = torch.full((n,), -7, dtype=torch.int32, device="cuda")
            objects = eng.group(dev64(keys), rep)
            assert objects == oobj, name
            assert (rep.cpu().numpy().astype(np.uint32) == orep).all(), name
            vals = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
            out = torch.empty(n, dtype=torch.int32, device="cuda")
            objects = eng.group_min(dev64(keys), torch.from_numpy(vals.view(np.int32)).cuda(), out)
            uniq, inv = np.unique(keys, return_inverse=True)
            mins = np.full(len(uniq), 0xFFFFFFFF, dtype=np.uint32)
            np.minimum.at(mins, inv, vals)
            assert objects == len(uniq) and (out.cpu().numpy().view(np.uint32) == mins[inv]).all(), name
        finally:
            eng.set_group_method()
        ko = torch.empty(n, dtype=torch.int64, device="cuda")
        vo = torch.empty(n, dtype=torch.int32, device="cuda")
        eng.sort_pairs(dev64(keys), None, ko, vo)
        rep2 = torch.full((n,), -7, dtype=torch.int32, device="cuda")
        assert eng.group_sorted(ko, vo, rep2) == oobj, name
        assert (rep2.cpu().numpy().astype(np.uint32) == orep).all(), name


@pytest.mark.parametrize("quanta", [1, 2, 3])
def test_hash_group_fused_vs_standalone(eng, oracle, quanta):
    """sd_cas_hash_group_sampled_dev (K1G: K1 with the grouping partition in its epilogue, then
    one bucket-table launch over the fixed-capacity regions): keys == K1's, rep and Objects ==
    the standalone grouping's, on 30 %-duplicate batches of 1, 2 (512-lane grid) and 3
    (256-lane grid) quanta; async use leaves the overflow flag 0; oracle parity on a sample."""
    q = eng.batch_quantum
    n = quanta * q
    content = torch.empty((n, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
    sizes = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_sampled(61 + quanta, 0, n, content, sizes, SAMPLED_CONTENT_LEN, dup_permille=300)
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    rep = torch.empty(n, dtype=torch.int32, device="cuda")
    keys2 = torch.zeros(n, dtype=torch.int64, device="cuda")
    rep2 = torch.zeros(n, dtype=torch.int32, device="cuda")
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    eng.hash_sampled(content, sizes, keys)
    objects = eng.group(keys, rep)
    assert eng.hash_group_sampled(content, sizes, keys2, rep2, ovf, want_objects=False) is None
    torch.cuda.synchronize()
    assert int(ovf.item()) == 0
    assert torch.equal(keys, keys2) and torch.equal(rep, rep2)
    out = torch.empty(1, dtype=torch.int64, device="cuda")
    eng._check(eng.L.sd_cas_copy_objects_dev(eng.h, out.data_ptr(), eng.stream), "copy_objects")
    torch.cuda.synchronize()
    assert int(out.item()) == objects
    # blocking form, twice (the region cursors are left zero by each call)
    for _ in range(2):
        rep2.zero_()
        assert eng.hash_group_sampled(content, sizes, keys2, rep2, ovf) == objects
        assert torch.equal(rep, rep2)
    rng = np.random.default_rng(quanta)
    idx = rng.integers(0, n, 200)
    host = content[torch.from_numpy(idx).cuda()].cpu().numpy()
    hs = sizes.cpu().numpy().view(np.uint64)[idx]
    want = oracle.cas_keys_strided(host.reshape(-1), SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN, hs)
    assert (keys2.cpu().numpy().view(np.uint64)[idx] == want).all()
    orep, oobj = oracle.group_canonical(keys2.cpu().numpy().view(np.uint64))
    assert oobj == objects and (rep2.cpu().numpy().astype(np.uint32) == orep).all()
    del content
    torch.cuda.empty_cache()


def test_hash_regions_split_pipelined(eng, oracle):
    """The fused chain's two halves as a pipelining caller uses them: batch i's bucket tables
    on a side stream while batch i+1 hashes into the other region set (the library orders a
    set's refill after its tables), a batch hashed but never grouped (its set's cursors must
    not leak into the next batch), and the async Object count via copy_objects — every rep ==
    the standalone grouping's."""
    q = eng.batch_quantum
    n = 2 * q
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    batches = []
    for j in range(4):
        content = torch.empty((n, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
        sizes = torch.empty(n, dtype=torch.int64, device="cuda")
        eng.synth_sampled(80 + j, j * n, n, content, sizes, SAMPLED_CONTENT_LEN, dup_permille=300)
        batches.append((content, sizes))
    torch.cuda.synchronize()
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    keys = [torch.empty(n, dtype=torch.int64, device="cuda") for _ in range(4)]
    reps = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(4)]
    objs = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(4)]
    done = []
    for j, (content, sizes) in enumerate(batches):
        eng.hash_regions_sampled(content, sizes, keys[j], reps[j], ovf, stream=main.cuda_stream)
        if j == 1:
            continue  # hashed, never grouped: dropped by the next hash_regions
        ev = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        eng.group_regions(n, reps[j], stream=side.cuda_stream, want_objects=False)
        eng._check(eng.L.sd_cas_copy_objects_dev(eng.h, objs[j].data_ptr(), side.cuda_stream), "copy")
        done.append(j)
    torch.cuda.synchronize()
    assert int(ovf.item()) == 0
    with pytest.raises(Exception):  # the last batch is grouped already
        eng.group_regions(n, reps[3])
    for j in done:
        rep = torch.empty(n, dtype=torch.int32, device="cuda")
        objects = eng.group(keys[j], rep)
        assert torch.equal(rep, reps[j]) and int(objs[j].item()) == objects, j
    kh = keys[0].cpu().numpy().view(np.uint64)
    orep, oobj = oracle.group_canonical(kh)
    assert (reps[0].cpu().numpy().astype(np.uint32) == orep).all() and oobj == int(objs[0].item())
    del batches
    torch.cuda.empty_cache()


@pytest.mark.parametrize("hot", [[20_000], [9_000, 7_000, 5_000, 3_000], []])
def test_hash_group_fused_overflow_and_fallback(eng, oracle, hot):
    """Coarse buckets outgrowing their fixed regions (files copied thousands of times in a
    batch of one quantum: region capacity ~450 rows): the flag is raised and the grouping is
    still exact — the async call's rep and Object count (copy_objects) equal the standalone
    grouping's with no caller regroup (each full region's table workgroup reads the region's
    rows and then its rows on the set's spill list into the same LDS table; the whole-key-array
    regroup behind it is forced in test_hash_group_fused_table_overflow_paths).  A batch that
    is not a multiple of the quantum runs K1 + the standalone chain (flag untouched)."""
    q = eng.batch_quantum
    for n in ([q, q + 1000] if not hot else [q]):
        content = torch.empty((n, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
        sizes = torch.empty(n, dtype=torch.int64, device="cuda")
        eng.synth_sampled(71, 0, n, content, sizes, SAMPLED_CONTENT_LEN, dup_permille=100)
        at = 1
        for h, copies in enumerate(hot):
            src = 40_000 + h  # the hot file's copies spread over the batch
            idx = torch.from_numpy(np.random.default_rng(h).choice(
                np.setdiff1d(np.arange(n), [40_000 + j for j in range(len(hot))]), copies,
                replace=False)).cuda()
            content[idx] = content[src].clone()
            sizes[idx] = sizes[src].clone()
            at += copies
        keys = torch.empty(n, dtype=torch.int64, device="cuda")
        rep = torch.empty(n, dtype=torch.int32, device="cuda")
        eng.hash_sampled(content, sizes, keys)
        objects = eng.group(keys, rep)
        keys2 = torch.empty(n, dtype=torch.int64, device="cuda")
        rep2 = torch.empty(n, dtype=torch.int32, device="cuda")
        ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
        eng.hash_group_sampled(content, sizes, keys2, rep2, ovf, want_objects=False)
        out = torch.zeros(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()  # (its zero fill, on torch's stream, before ours writes it)
        eng._check(eng.L.sd_cas_copy_objects_dev(eng.h, out.data_ptr(), eng.stream), "copy_objects")
        torch.cuda.synchronize()
        assert torch.equal(keys, keys2)
        assert int(ovf.item()) == (1 if hot else 0)
        assert torch.equal(rep, rep2) and int(out.item()) == objects
        rep2.zero_()
        ovf.zero_()
        assert eng.hash_group_sampled(content, sizes, keys2, rep2, ovf) == objects
        assert torch.equal(rep, rep2)
        orep, oobj = oracle.group_canonical(keys.cpu().numpy().view(np.uint64))
        assert oobj == objects and (rep.cpu().numpy().astype(np.uint32) == orep).all()
        del content
        torch.cuda.empty_cache()


@pytest.mark.parametrize("hot", [[20_000], [9_000, 7_000, 5_000], []])
def test_hash_group_fused_table_overflow_paths(eng, oracle, monkeypatch, hot):
    """the fused chain's table overflow paths, which uniform BLAKE3 keys never
    reach (a region holds ~5,100 distinct keys at 1.31 M files against a 10,752 bound, and K1G
    keys cannot be crafted): a context created with SD_CAS_TEST_TABLE_FILL=200 sends every
    region with more than 200 distinct keys to its own global table, and a FULL region (hot
    files copied thousands of times: its rows + spill list) to the regroup from the whole key
    array in a global table carved from the set's overflow slots — several hot files carve
    several tables, and K1G's keys must stay alive until the tables finish.  rep and Objects
    == the standalone grouping and the oracle, over both region sets."""
    from spacedrive_amd import CasEngine
    monkeypatch.setenv("SD_CAS_TEST_TABLE_FILL", "200")
    e2 = CasEngine(0)
    q = eng.batch_quantum
    n = q
    content = torch.empty((n, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
    sizes = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_sampled(72, 0, n, content, sizes, SAMPLED_CONTENT_LEN, dup_permille=100)
    for h, copies in enumerate(hot):
        idx = torch.from_numpy(np.random.default_rng(10 + h).choice(
            np.setdiff1d(np.arange(n), [40_000 + j for j in range(len(hot))]), copies,
            replace=False)).cuda()
        content[idx] = content[40_000 + h].clone()
        sizes[idx] = sizes[40_000 + h].clone()
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    rep = torch.empty(n, dtype=torch.int32, device="cuda")
    eng.hash_sampled(content, sizes, keys)
    objects = eng.group(keys, rep)
    orep, oobj = oracle.group_canonical(keys.cpu().numpy().view(np.uint64))
    assert oobj == objects and (rep.cpu().numpy().astype(np.uint32) == orep).all()
    for rnd in range(3):  # the two region sets alternate
        keys2 = torch.empty(n, dtype=torch.int64, device="cuda")
        rep2 = torch.empty(n, dtype=torch.int32, device="cuda")
        ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        got = e2.hash_group_sampled(content, sizes, keys2, rep2, ovf)
        assert torch.equal(keys, keys2), rnd
        assert got == objects and torch.equal(rep, rep2), rnd
        assert int(ovf.item()) == (1 if hot else 0)
    e2.close()
    del content
    torch.cuda.empty_cache()


def test_hash_regions_streams_and_ungrouped(eng):
    """K1G batches on two streams with one batch hashed but never grouped — the
    next hash_regions into its set waits for that K1G (no cursor or row corruption), tables on
    a third stream wait for their own K1G, and the Object count of the last grouping survives
    the refill of its set (copy_objects after it)."""
    q = eng.batch_quantum
    n = q
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    data = []
    for j in range(5):
        c = torch.empty((n, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
        z = torch.empty(n, dtype=torch.int64, device="cuda")
        eng.synth_sampled(300 + j, j * n, n, c, z, SAMPLED_CONTENT_LEN, dup_permille=300)
        data.append((c, z))
    torch.cuda.synchronize()
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    keys = [torch.empty(n, dtype=torch.int64, device="cuda") for _ in range(5)]
    reps = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(5)]
    obj = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(5)]
    late = torch.zeros(1, dtype=torch.int64, device="cuda")
    # torch's zero fills run on its current stream, not on s1/s2/s3: they must be complete
    # before the library writes these tensors on those streams — the caller-side ordering rule
    # of include/sd_hip_cas.h's conventions and INTEGRATION.md §1 (round 4's failure of this
    # test was exactly a missing synchronize here)
    torch.cuda.synchronize()
    # batch 0 on s1 (grouped on s3), batch 1 on s2 never grouped, batch 2 on s1 refills set 0,
    # batch 3 on s2 refills batch 1's set while its K1G may still run; batch 4 grouped last
    plan = [(s1, True), (s2, False), (s1, True), (s2, True), (s1, True)]
    for j, ((c, z), (st, grp)) in enumerate(zip(data, plan)):
        eng.hash_regions_sampled(c, z, keys[j], reps[j], ovf, stream=st.cuda_stream)
        if grp:
            eng.group_regions(n, reps[j], stream=s3.cuda_stream, want_objects=False)
            eng._check(eng.L.sd_cas_copy_objects_dev(eng.h, obj[j].data_ptr(), s3.cuda_stream), "copy")
    torch.cuda.synchronize()
    for j in (0, 2, 3, 4):
        rep = torch.empty(n, dtype=torch.int32, device="cuda")
        assert eng.group(keys[j], rep) == int(obj[j].item()) and torch.equal(rep, reps[j]), j
    # batch 4's count lives in its region set; two more hash_regions (never grouped) refill
    # that set: copy_objects still returns batch 4's count
    eng.hash_regions_sampled(data[0][0], data[0][1], keys[0], reps[0], ovf, stream=s1.cuda_stream)
    eng.hash_regions_sampled(data[1][0], data[1][1], keys[1], reps[1], ovf, stream=s2.cuda_stream)
    eng._check(eng.L.sd_cas_copy_objects_dev(eng.h, late.data_ptr(), s3.cuda_stream), "copy")
    torch.cuda.synchronize()
    assert int(late.item()) == int(obj[4].item())
    del data
    torch.cuda.empty_cache()


def test_workspace_ordered_across_streams(eng, oracle):
    """One context, device calls on two streams with no host sync between them: grouping,
    group_min and the packed hash's length sort share the context workspace, which the
    library orders across streams (an event per use)."""
    rng = np.random.default_rng(71)
    n = 400_000
    ka = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
    ka[1::3] = ka[0::3][: len(ka[1::3])]
    kb = rng.integers(0, 2 ** 62, n, dtype=np.uint64)
    kb[::2] = kb[1::2]
    vb = rng.integers(0, 2 ** 31, n, dtype=np.uint64).astype(np.int32)
    da, db, dvb = dev64(ka), dev64(kb), torch.from_numpy(vb).cuda()
    sz = torch.empty(50_000, dtype=torch.int64, device="cuda")
    ln = torch.empty(50_000, dtype=torch.int32, device="cuda")
    of = torch.empty(50_000, dtype=torch.int64, device="cuda")
    nb = eng.synth_small(72, 0, 50_000, sz, ln, of, None)
    arena = torch.empty(nb + 64, dtype=torch.uint8, device="cuda")
    eng.synth_small(72, 0, 50_000, sz, ln, of, arena)
    want_p = torch.empty(50_000, dtype=torch.int64, device="cuda")
    eng.set_latency_threshold(0, 0)  # K2 with its on-device length sort (workspace)
    try:
        eng.hash_packed(arena, of, ln, sz, want_p)
        torch.cuda.synchronize()
        orep_a, _ = oracle.group_canonical(ka)
        uniq, inv = np.unique(kb, return_inverse=True)
        mins = np.full(len(uniq), 2 ** 31, dtype=np.int64)
        np.minimum.at(mins, inv, vb.astype(np.int64))
        s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
        for trial in range(4):
            ra = torch.empty(n, dtype=torch.int32, device="cuda")
            rb = torch.empty(n, dtype=torch.int32, device="cuda")
            kp = torch.empty(50_000, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            with torch.cuda.stream(s1):
                eng.group(da, ra, want_objects=False)
            with torch.cuda.stream(s2):
                eng.group_min(db, dvb, rb, want_objects=False)
            with torch.cuda.stream(s3):
                eng.hash_packed(arena, of, ln, sz, kp)
            torch.cuda.synchronize()
            assert (ra.cpu().numpy().astype(np.uint32) == orep_a).all(), trial
            assert (rb.cpu().numpy() == mins[inv]).all(), trial
            assert torch.equal(kp, want_p), trial
    finally:
        eng.set_latency_threshold()


def test_group_min_vs_numpy(eng):
    rng = np.random.default_rng(41)
    for n, pool in [(1, 1), (777, 100), (250_000, 90_000), (2_000_000, 1_500_000)]:
        base = rng.integers(0, 2 ** 64, pool, dtype=np.uint64)
        keys = base[rng.integers(0, pool, n)]
        vals = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        objects = eng.group_min(dev64(keys), torch.from_numpy(vals.view(np.int32)).cuda(), out)
        uniq, inv = np.unique(keys, return_inverse=True)
        mins = np.full(len(uniq), 0xFFFFFFFF, dtype=np.uint32)
        np.minimum.at(mins, inv, vals)
        assert objects == len(uniq)
        assert (out.cpu().numpy().view(np.uint32) == mins[inv]).all()


@pytest.mark.parametrize("n_uni", [900_000, 2_400_000])
def test_group_regions_overflow(eng, oracle, n_uni):
    """The region chains: up to 1.44M keys sd_region_partition into 256 fixed-capacity regions
    + sd_bucket_min_regions_keys (a region past capacity regrouped from the whole input);
    above, sd_region_partition_big + sd_part_refine_regions + the fine tables (rows past a
    region's capacity through the spill list).  Regions pushed past capacity — one key
    repeated 300K times, and 3 regions each given 20K crafted distinct keys — plus a uniform
    30 %-duplicate batch; sd_cas_group vs the oracle and sd_cas_group_min (random u32 vals) vs
    numpy, twice in a row (the region cursors are left zero)."""
    rng = np.random.default_rng(43)
    crafted = []
    for top in (3, 77, 200):  # mixed top byte = the region (2^8 coarse regions at these sizes)
        low = rng.integers(0, 2 ** 56, 20_000, dtype=np.uint64)
        crafted.append(np.array([unmix64((top << 56) | int(x)) for x in low], dtype=np.uint64))
    uni = rng.integers(0, 2 ** 64, n_uni, dtype=np.uint64)
    cases = {
        "one key x300K": np.concatenate([uni, np.full(300_000, 0x1234567, dtype=np.uint64)]),
        "3 crafted regions": np.concatenate([uni] + crafted),
        "uniform 30% dup": uni[rng.integers(0, int(n_uni * 0.7), int(n_uni * 1.2))],
    }
    for name, keys in cases.items():
        keys = keys[rng.permutation(len(keys))]
        n = len(keys)
        for _ in range(2):
            rep = torch.empty(n, dtype=torch.int32, device="cuda")
            objects = eng.group(dev64(keys), rep)
            orep, oobj = oracle.group_canonical(keys)
            assert objects == oobj, name
            assert (rep.cpu().numpy().astype(np.uint32) == orep).all(), name
        vals = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        objects = eng.group_min(dev64(keys), torch.from_numpy(vals.view(np.int32)).cuda(), out)
        uniq, inv = np.unique(keys, return_inverse=True)
        mins = np.full(len(uniq), 0xFFFFFFFF, dtype=np.uint32)
        np.minimum.at(mins, inv, vals)
        assert objects == len(uniq), name
        assert (out.cpu().numpy().view(np.uint32) == mins[inv]).all(), name


def test_partition_range_vs_numpy(eng):
    from tests.test_shard_cpu import range_part
    rng = np.random.default_rng(42)
    for n, parts in [(0, 3), (1, 1), (1000, 2), (123_457, 3), (1 << 20, 8), (50_000, 7)]:
        keys = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
        if n >= 8:
            keys[:8] = [0, 1, 2 ** 63 - 1, 2 ** 63, 2 ** 64 - 1, -((-(1 << 64)) // 3), (1 << 64) // 3, 5]
        ko = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
        po = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
        counts = torch.empty(parts, dtype=torch.int64, device="cuda")
        eng.partition(dev64(keys) if n else torch.empty(0, dtype=torch.int64, device="cuda"),
                      parts, ko, po, counts)
        want = np.bincount(range_part(keys, parts), minlength=parts)
        assert counts.cpu().tolist() == want.tolist()
        if n == 0:
            continue
        k, p = host64(ko)[:n], po.cpu().numpy()[:n]
        assert (np.sort(p) == np.arange(n)).all() and (keys[p] == k).all()
        assert (np.diff(range_part(k, parts)) >= 0).all()  # part-contiguous in part order


CHECKSUM_LENS = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 4097, 255 * 1024, 256 * 1024,
                 256 * 1024 + 1, 257 * 1024 + 3, 512 * 1024, 65536 * 1024 + 5, 3 * 256 * 1024 * 256 + 777]


def test_device_blake3_runs_the_reference_balloon(eng, oracle):
    """The device BLAKE3 (sd_cas_checksum_dev, K3) driven through the reference's password
    hash — Balloon::<blake3::Hasher> (crates/crypto/src/keys/hashing.rs:95-114; every block
    hash a streamed 40-106-B, one- or two-block input) — at s_cost 256, t_cost 2, with and
    without the KAT's secret, equals the oracle's Balloon, whose full-size runs reproduce the
    reference's six HASH_B3BALLOON KATs (tests/test_oracle.py): the GPU's compression,
    flags and block chaining sit on the same reference vectors as the oracle's.  Sequential
    by construction: 5,376 dependent device hashes per run."""
    buf = torch.zeros(256, dtype=torch.uint8, device="cuda")

    def H(*parts):
        m = b"".join(parts)
        buf[:len(m)].copy_(torch.frombuffer(bytearray(m), dtype=torch.uint8))
        return bytes.fromhex(eng.checksum_dev(buf, len(m)))

    def le(v):
        return int(v).to_bytes(8, "little")

    pwd, salt = b"password", b"\xff" * 16
    for secret in (None, b"\x55" * 18):
        sec = secret or b""
        s_cost, t_cost, cnt = 256, 2, 0
        blk = [H(le(cnt), pwd, salt, sec)]
        cnt += 1
        for m in range(1, s_cost):
            blk.append(H(le(cnt), blk[m - 1]))
            cnt += 1
        for t in range(t_cost):
            for m in range(s_cost):
                blk[m] = H(le(cnt), blk[m - 1], blk[m])  # blk[-1] is the last block for m == 0
                cnt += 1
                for i in range(3):
                    idx = H(le(t), le(m), le(i))
                    other = int.from_bytes(H(le(cnt), salt, sec, idx), "little") % s_cost
                    cnt += 1
                    blk[m] = H(le(cnt), blk[m], blk[other])
                    cnt += 1
        assert blk[-1] == oracle.balloon_blake3(pwd, salt, secret, s_cost, t_cost), secret is not None


def test_device_kernels_vs_independent_c_blake3(eng, tmp_path):
    """The product's kernels against the BLAKE3 team's C implementation (1.8.2, exported by
    ROCm's libclang-cpp.so; tests/ext_blake3.py) with no oracle in between: K1 (8,192 sampled
    files), K2 (140,000 ragged whole-file messages: above the two-quanta crossover), the
    latency path (3,000 whole files through the host entry), K3 (one 1 GiB + 7 device
    buffer), K3b (a validator batch of small, mid and multi-MiB buffers) and the streamed
    file path (a 300 MB file, one call and the batch call)."""
    from tests import ext_blake3 as ext
    if not ext.available():
        pytest.skip("no libclang-cpp.so with the BLAKE3 C API in this image")
    rng = np.random.default_rng(91)
    # K1
    n = 8192
    content = rng.integers(0, 256, (n, SAMPLED_CONTENT_LEN), dtype=np.uint8)
    sizes = rng.integers(MINIMUM_FILE_SIZE + 1, 2 ** 40, n, dtype=np.uint64)
    keys = torch.zeros(n, dtype=torch.int64, device="cuda")
    eng.hash_sampled(torch.from_numpy(content).cuda(), dev64(sizes), keys)
    want = np.array([ext.cas_key(content[i], int(sizes[i])) for i in range(n)], dtype=np.uint64)
    assert (host64(keys) == want).all()
    # K2
    lens = rng.integers(1, 8193, 140_000)
    lens[:64] = [1, 63, 64, 65, 1016, 1017, 1024, 1025] * 8
    arena = rng.integers(0, 256, int(((lens + 15) // 16 * 16).sum()) + 128, dtype=np.uint8)
    offs = np.zeros(len(lens), dtype=np.uint64)
    offs[1:] = np.cumsum((lens[:-1] + 15) // 16 * 16)
    keys = torch.zeros(len(lens), dtype=torch.int64, device="cuda")
    eng.hash_packed(torch.from_numpy(arena).cuda(), dev64(offs),
                    torch.from_numpy(lens.astype(np.int32)).cuda(), dev64(lens.astype(np.uint64)), keys)
    want = np.array([ext.cas_key(arena[int(o):int(o) + int(L)], int(L)) for o, L in zip(offs, lens)],
                    dtype=np.uint64)
    assert (host64(keys) == want).all()
    # latency path, host entry
    items = [(rng.integers(0, 256, int(L), dtype=np.uint8).tobytes(), int(L))
             for L in rng.integers(1, MINIMUM_FILE_SIZE + 1, 3000)]
    got = eng.generate_cas_keys(items)
    assert [int(x) for x in got] == [ext.cas_key(c, L) for c, L in items]
    # K3: one device buffer
    big = torch.randint(0, 256, ((1 << 30) + 7,), dtype=torch.uint8, device="cuda")
    assert eng.checksum_dev(big) == ext.blake3(big.cpu().numpy()).hex()
    del big
    # K3b: a validator batch
    blens = np.concatenate([rng.integers(0, 16_385, 200), rng.integers(16_385, 2 << 20, 80),
                            rng.integers(2 << 20, 40 << 20, 12)])
    boffs = np.zeros(len(blens), dtype=np.int64)
    boffs[1:] = np.cumsum((blens[:-1] + 15) // 16 * 16)
    barena = torch.randint(0, 256, (int(boffs[-1] + blens[-1]) + 16,), dtype=torch.uint8, device="cuda")
    out = torch.zeros((len(blens), 32), dtype=torch.uint8, device="cuda")
    eng.checksums_dev(barena, torch.from_numpy(boffs).cuda(), torch.from_numpy(blens.astype(np.int64)).cuda(), out)
    h = barena.cpu().numpy()
    got = out.cpu().numpy()
    for i, (o, L) in enumerate(zip(boffs, blens)):
        assert got[i].tobytes() == ext.blake3(h[int(o):int(o) + int(L)]), (i, int(L))
    # streamed file path
    f = tmp_path / "big.bin"
    data = rng.integers(0, 256, 300_000_123, dtype=np.uint8)
    data.tofile(f)
    want = ext.blake3(data).hex()
    assert eng.file_checksum(str(f)) == want
    digests, errs = eng.file_checksums([str(f)])
    assert digests == [want] and int(errs[0]) == 0


def test_device_trees_on_the_independently_pinned_lengths(eng, oracle):
    """The lengths whose trees hf_xet's BLAKE3 pins in the oracle (tests/golden/xet_blake3.json,
    1-128 chunks): the same contents through the product's three whole-message kernels — the
    validator batch (K3b), the single-buffer tree (K3) and the whole-file cas_id (K2, message
    le64(size) || content) — bit-exact against the oracle."""
    import json
    import torch
    from tests.golden.make_xet_vectors import content
    with open(os.path.join(os.path.dirname(__file__), "golden", "xet_blake3.json")) as f:
        vecs = json.load(f)["vectors"]
    datas = [content(v["len"], v["seed"]) for v in vecs]
    offs = np.zeros(len(datas), np.int64)
    pos = 0
    for i, d in enumerate(datas):
        offs[i] = pos
        pos += (len(d) + 15) // 16 * 16
    arena = np.zeros(pos, np.uint8)
    for o, d in zip(offs, datas):
        arena[o:o + len(d)] = np.frombuffer(d, np.uint8)
    lens = np.array([len(d) for d in datas], np.int64)
    out = torch.zeros((len(datas), 32), dtype=torch.uint8, device="cuda")
    eng.checksums_dev(torch.from_numpy(arena).cuda(), torch.from_numpy(offs).cuda(),
                      torch.from_numpy(lens).cuda(), out)
    got = out.cpu().numpy()
    for i, d in enumerate(datas):
        want = oracle.blake3(d)
        assert got[i].tobytes() == want, len(d)
        if i % 7 == 0:
            assert eng.checksum_dev(torch.from_numpy(np.frombuffer(d, np.uint8).copy()).cuda()) == want.hex()
    small = [(d, len(d)) for d in datas if len(d) <= 102_400]
    assert eng.generate_cas_ids(small) == [oracle.cas_id(d, n) for d, n in small]


def test_device_blake3_reproduces_reference_balloon_kats(eng, golden):
    """The reference's own Balloon-BLAKE3 known answers, computed on the GPU: the product's
    device BLAKE3 compression (spacedrive_amd/csrc/blake3_device.hpp) driven through
    Balloon::<blake3::Hasher> (tests/native/balloon_dev.hip, the construction of
    oracle/balloon_ref.c) reproduces HASH_B3BALLOON_EXPECTED[0] and
    HASH_B3BALLOON_WITH_SECRET_EXPECTED[0] (crates/crypto/src/keys/hashing.rs:180-208,
    s_cost 131,072, t_cost 2): ~2.75 M dependent one- and two-block hashes per chain, the
    two chains side by side.  The GPU thereby sits on the reference's vectors directly, not
    only on the oracle's outputs."""
    lib_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libballoon_dev.so")
    assert os.path.exists(lib_path), "build() builds tests/native/libballoon_dev.so"
    L = ctypes.CDLL(lib_path)
    L.balloon_dev_run.restype = ctypes.c_int
    g = golden["balloon_b3_kat"]
    pwd, salt, sec = (bytes.fromhex(g[k]) for k in ("password_hex", "salt_hex", "secret_hex"))
    secrets = (ctypes.c_char_p * 2)(b"", sec)
    lens = (ctypes.c_uint32 * 2)(0, len(sec))
    out = ctypes.create_string_buffer(64)
    rc = L.balloon_dev_run(pwd, ctypes.c_uint32(len(pwd)), salt, ctypes.c_uint32(len(salt)), secrets,
                           lens, ctypes.c_int(2), ctypes.c_uint64(131_072), ctypes.c_uint64(2), out)
    assert rc == 0
    want = {v["secret"]: v["expected_hex"] for v in g["vectors"] if v["s_cost"] == 131_072}
    assert out.raw[:32].hex() == want[False]
    assert out.raw[32:].hex() == want[True]


def test_checksum_device_vs_oracle(eng, oracle):
    rng = np.random.default_rng(7)
    for L in CHECKSUM_LENS:
        d = rng.integers(0, 256, L, dtype=np.uint8)
        buf = torch.zeros(L + 16, dtype=torch.uint8, device="cuda")
        buf[:L] = torch.from_numpy(d).cuda()
        assert eng.checksum_dev(buf, L) == oracle.blake3(d.tobytes()).hex(), L


def test_file_checksum_streamed(eng, oracle, tmp_path):
    import spacedrive_amd as sd
    rng = np.random.default_rng(8)
    for L in [0, 1, 1 << 20, (64 << 20) - 1, (64 << 20), (64 << 20) + 1, (2 * 64 << 20) + 12345]:
        p = tmp_path / f"v{L}"
        p.write_bytes(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        assert eng.file_checksum(str(p)) == oracle.file_checksum(str(p)), L
        p.unlink()
    with pytest.raises(OSError):
        sd.file_checksum(str(tmp_path / "nope"))


ORC_THREADS = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)


def test_checksum_device_over_4gib(eng, oracle):
    """BASELINE config 5 sizes on the device path: buffers past 4 GiB with odd tails — byte
    offsets above 2^32, chunk counters above 2^22, and the multi-level CV reduce (> 256 x 256
    1 MiB subtrees) — vs the oracle's tree-parallel hash of the same generated stream."""
    for L in [(4 << 30) + 777, (5 << 30) + (1 << 20) + 3]:
        buf = torch.empty(L + 64, dtype=torch.uint8, device="cuda")
        eng.synth_stream(55, 3, 0, L, buf)
        # the device generator is the oracle's stream, at the start and past 2^32
        for off in (0, (L - 4096) & ~7):  # the last window lies past 2^32
            assert (buf[off:off + 4096].cpu().numpy() == oracle.fill_content_range(55, 3, off, 4096)).all()
        got = eng.checksum_dev(buf, L)
        assert got == oracle.stream_blake3_mt(55, 3, L, ORC_THREADS).hex(), L
        from tests import ext_blake3 as ext
        if ext.available():  # and the BLAKE3 team's C implementation on the same bytes
            assert got == ext.blake3(buf[:L].cpu().numpy()).hex(), L
        del buf
        torch.cuda.empty_cache()


def test_file_checksum_streamed_multi_gib(eng, oracle, tmp_path):
    """file_checksum (hash.rs:11-25) of a > 4 GiB file streamed from tmpfs through the
    pinned 64 MiB segments: 65 segment subtrees + the GPU CV reduce, vs the oracle (the
    generated stream and the file read back, tree-parallel)."""
    L = (4 << 30) + 12345
    d = "/dev/shm" if os.path.isdir("/dev/shm") else str(tmp_path)
    path = os.path.join(d, f"sdcas_checksum_{os.getpid()}.bin")
    try:
        with open(path, "wb") as fh:
            piece = 256 << 20
            for off in range(0, L, piece):
                fh.write(oracle.fill_content_range(56, 4, off, min(piece, L - off)).tobytes())
        want = oracle.stream_blake3_mt(56, 4, L, ORC_THREADS).hex()
        assert eng.file_checksum(path) == want
        assert oracle.file_checksum_mt(path, ORC_THREADS) == want
        from tests import ext_blake3 as ext
        if ext.available():  # the file's bytes through the BLAKE3 team's C implementation
            assert ext.blake3(np.memmap(path, dtype=np.uint8, mode="r")).hex() == want
    finally:
        if os.path.exists(path):
            os.unlink(path)


def test_file_checksum_reads_to_eof(eng, oracle):
    """hash.rs:15-21 hashes what the reads return until the first short read, not st_size: a
    procfs file whose st_size is 0 but which has content is hashed over that content."""
    p = "/proc/sys/kernel/ostype"
    if not os.path.exists(p) or os.stat(p).st_size != 0:
        pytest.skip("no procfs file with st_size 0")
    assert eng.file_checksum(p) == oracle.file_checksum(p) == oracle.blake3(open(p, "rb").read()).hex()


def _short_read_files():
    """procfs seq_files whose first 1 MiB read() returns less than the whole file (about one
    page): hash.rs:15-21 stops there.  Returns [(path, first read, rest)]."""
    out = []
    for p in ("/proc/self/mountinfo", "/proc/kallsyms", "/proc/self/mounts"):
        try:
            fd = os.open(p, os.O_RDONLY)
        except OSError:
            continue
        try:
            first = os.read(fd, 1 << 20)
            rest = os.read(fd, 1 << 20)
        finally:
            os.close(fd)
        if 0 < len(first) < (1 << 20) and rest:
            out.append((p, first, rest))
    return out


def test_file_checksum_short_reads(eng, oracle):
    """hash.rs:15-21 issues 1 MiB reads and stops after the FIRST short one.  A procfs
    seq_file returns about one page per read, so the reference hashes only that page — and
    so must both entry points (sd_cas_file_checksum and the batched sd_cas_file_checksums'
    redo path), vs the oracle's literal read loop on the same file."""
    files = _short_read_files()
    if not files:
        pytest.skip("no procfs seq_file longer than one read")
    for p, first, rest in files[:2]:
        want = oracle.file_checksum(p)
        assert want == oracle.blake3(first).hex(), p  # the literal loop hashed one read
        assert want != oracle.blake3(first + rest).hex()
        assert eng.file_checksum(p) == want, p
        digests, errs = eng.file_checksums([p, "/proc/sys/kernel/ostype", p])
        assert list(errs) == [0, 0, 0]
        assert digests[0] == digests[2] == want, p


def test_file_checksum_fifo(eng, oracle, tmp_path):
    """A FIFO is not a regular file: its reads return what the writer has written so far.
    The writer puts 4,000 bytes (< PIPE_BUF: one atomic write), waits, then writes more; the
    first 1 MiB read returns the 4,000 bytes and hash.rs:15-21 stops there — both entry
    points must hash exactly those bytes."""
    import threading
    import time
    rng = np.random.default_rng(32)
    a = rng.integers(0, 256, 4000, dtype=np.uint8).tobytes()
    b = rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes()
    want = oracle.blake3(a).hex()
    for entry in ("one", "batch"):
        fifo = str(tmp_path / f"fifo_{entry}")
        os.mkfifo(fifo)

        def writer():
            try:
                with open(fifo, "wb", buffering=0) as fh:
                    fh.write(a)
                    time.sleep(0.5)
                    fh.write(b)
            except BrokenPipeError:
                pass  # the reader stopped after its first short read
        t = threading.Thread(target=writer, daemon=True)
        t.start()
        if entry == "one":
            got = eng.file_checksum(fifo)
        else:
            digests, errs = eng.file_checksums([fifo])
            assert errs[0] == 0
            got = digests[0]
        t.join(5)
        assert got == want, entry


def test_checksums_batch_dev_vs_oracle(eng, oracle):
    """The validator over many buffers in one launch chain (sd_cas_checksums_dev): ragged
    lengths around every chunk / 1 MiB-subtree boundary, a 300 MiB buffer (> 256 subtree CVs:
    the two-level in-LDS reduce), buffers in shuffled arena order, vs the oracle per buffer."""
    rng = np.random.default_rng(9)
    lens = (CHECKSUM_LENS[:-1] + [(1 << 20) - 1, 1 << 20, (1 << 20) + 1, (256 << 20) + 4097,
                                  (300 << 20) + 5, 5 * (1 << 20) + 17]
            + [int(x) for x in rng.integers(0, 3 << 20, 300)])
    order = rng.permutation(len(lens))
    offs = np.zeros(len(lens), dtype=np.uint64)
    o = 0
    for i in order:  # arena order != index order
        offs[i] = o
        o += (lens[i] + 15) // 16 * 16 + 16 * int(rng.integers(0, 3))
    arena_bytes = o + 16
    arena = torch.empty(arena_bytes, dtype=torch.uint8, device="cuda")
    seed = 91
    eng.synth_stream(seed, 1, 0, arena_bytes // 8 * 8, arena)
    host = arena.cpu().numpy()
    out = torch.zeros((len(lens), 32), dtype=torch.uint8, device="cuda")
    eng.checksums_dev(arena, dev64(offs), dev64(np.array(lens, dtype=np.uint64)), out)
    got = out.cpu().numpy()
    for i, L in enumerate(lens):
        want = oracle.blake3(host[int(offs[i]):int(offs[i]) + L].tobytes())
        assert got[i].tobytes() == want, (i, L)
    # buffers past arena_bytes or misaligned are refused, not read out of bounds
    with pytest.raises(Exception):
        eng.checksums_dev(arena, dev64(offs), dev64(np.array(lens, dtype=np.uint64)), out,
                          arena_bytes=1 << 20)
    bad_offs = offs.copy()
    bad_offs[3] += 8
    with pytest.raises(Exception):
        eng.checksums_dev(arena, dev64(bad_offs), dev64(np.array(lens, dtype=np.uint64)), out)
    # a valid call on the same context still works afterwards
    eng.checksums_dev(arena, dev64(offs), dev64(np.array(lens, dtype=np.uint64)), out)
    assert (out.cpu().numpy() == got).all()


@pytest.mark.parametrize("shape", ["uniform", "skewed"])
def test_checksums_batch_lane_path(eng, oracle, shape):
    """A batch of 140,000 buffers (>= LANE_MIN_BUFFERS: buffers of <= 128 chunks one per lane,
    sorted by chunk count): lengths at every chunk / block / quad boundary of the lane class
    (0, 1, 15, 16, 63, 64, 1023-1025, 64 and 128 KiB +-1), 128 KiB + 1 and larger buffers in
    the same batch (the mid and subtree kernels), an arena whose last buffer ends exactly at
    arena_bytes, shuffled arena order — every digest vs the oracle.  "uniform": lengths
    U(0, 128 KiB), every lane-class buffer goes one per lane; "skewed": ~96 % U(0, 1 KiB),
    1.5 % U(64, 128 KiB) and 3,500 of U(1, 64) KiB, so the tail cut (~13 chunks) leaves
    14..16-chunk buffers to sd_b3_batch_small16, 17..64 to small64 and 65..128 to mid, each
    walking its range of the sorted order, in the same chain."""
    rng = np.random.default_rng(12 if shape == "uniform" else 13)
    edge = [0, 1, 15, 16, 17, 63, 64, 65, 127, 128, 1023, 1024, 1025, 2047, 2048, 2049,
            (63 << 10) + 1, (64 << 10) - 1, 64 << 10, (64 << 10) + 1, (127 << 10) + 1,
            (128 << 10) - 1, 128 << 10, (128 << 10) + 1, (200 << 10) + 3, (3 << 20) + 11]
    n = 140_000
    if shape == "uniform":
        lens = rng.integers(0, 128 << 10, n).astype(np.int64)
        lens[rng.integers(0, n, 5000)] = rng.integers(0, 1100, 5000)  # one-chunk buffers
    else:
        lens = rng.integers(0, 1 << 10, n).astype(np.int64)
        long_ = rng.random(n) < 0.015
        lens[long_] = rng.integers(64 << 10, 128 << 10, int(long_.sum()))
        lens[rng.integers(0, n, 3500)] = rng.integers(1 << 10, 64 << 10, 3500)  # 2-64 chunks
    lens[: len(edge)] = edge
    lens[rng.integers(len(edge), n, 40)] = rng.integers(129 << 10, 2 << 20, 40)
    order = rng.permutation(n)
    offs = np.zeros(n, dtype=np.uint64)
    o = 0
    for i in order:
        offs[i] = o
        o += (int(lens[i]) + 15) // 16 * 16
    last = int(order[-1])
    arena_bytes = int(offs[last]) + int(lens[last])  # the last buffer ends at arena_bytes
    arena = torch.empty(o + 16, dtype=torch.uint8, device="cuda")
    eng.synth_stream(33, 2, 0, (o + 16) // 8 * 8, arena)
    host = arena.cpu().numpy()
    out = torch.zeros((n, 32), dtype=torch.uint8, device="cuda")
    eng.checksums_dev(arena, dev64(offs), dev64(lens.astype(np.uint64)), out,
                      arena_bytes=arena_bytes)
    got = out.cpu().numpy()
    bad = [i for i in range(n)
           if got[i].tobytes() != oracle.blake3(host[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes())]
    assert not bad, (len(bad), [(i, int(lens[i])) for i in bad[:8]])
    del arena
    torch.cuda.empty_cache()


def test_checksums_batch_overlapping_buffers_refused(eng, oracle):
    """The ABI does not forbid overlapping buffers, but their subtree work list can exceed
    the workspace sized from arena_bytes: such a batch is refused with EINVAL, never read
    out of bounds — including 4,194,305 buffers of (0, 1 GiB) in a 1 GiB arena, whose 2^32 +
    1,024 subtree groups wrap the u32 group scan to 1,024 (the wrapped total used
    to pass the check).  A valid call on the same context works afterwards."""
    G = 1 << 30
    arena = torch.empty(G + 64, dtype=torch.uint8, device="cuda")
    eng.synth_stream(58, 1, 0, 1 << 20, arena)
    for n, L in [(64, 64 << 20), (4_194_305, G)]:
        offs = torch.zeros(n, dtype=torch.int64, device="cuda")
        lens = torch.full((n,), L, dtype=torch.int64, device="cuda")
        out = torch.zeros((n, 32), dtype=torch.uint8, device="cuda")
        with pytest.raises(Exception, match="exceed"):
            eng.checksums_dev(arena, offs, lens, out, arena_bytes=G)
        del offs, lens, out
    offs = torch.tensor([0, 1 << 20], dtype=torch.int64, device="cuda")
    lens = torch.tensor([1 << 20, (3 << 20) + 5], dtype=torch.int64, device="cuda")
    out = torch.zeros((2, 32), dtype=torch.uint8, device="cuda")
    eng.checksums_dev(arena, offs, lens, out, arena_bytes=G)
    host = arena[:(4 << 20) + 5].cpu().numpy()
    assert bytes(out[0].cpu().numpy()) == oracle.blake3(host[:1 << 20].tobytes())
    assert bytes(out[1].cpu().numpy()) == oracle.blake3(host[1 << 20:(4 << 20) + 5].tobytes())
    del arena
    torch.cuda.empty_cache()


def test_checksums_batch_over_64k_items(eng, oracle):
    """Two 40 GiB buffers in one batch chain: 81,920 subtree work items, more than the
    65,536-workgroup grid, so the groups kernel strides; 160 reduce blocks per buffer; byte
    offsets past 2^32 — vs the oracle's tree-parallel hash of the same generated streams."""
    L = 40 << 30
    arena = torch.empty(2 * L + 64, dtype=torch.uint8, device="cuda")
    for f in range(2):
        eng.synth_stream(57, 10 + f, 0, L, arena[f * L:])
    offs = torch.tensor([0, L], dtype=torch.int64, device="cuda")
    lens = torch.tensor([L, L - 4096 - 5], dtype=torch.int64, device="cuda")
    out = torch.zeros((2, 32), dtype=torch.uint8, device="cuda")
    eng.checksums_dev(arena, offs, lens, out)
    got = [bytes(r).hex() for r in out.cpu().numpy()]
    assert got[0] == oracle.stream_blake3_mt(57, 10, L, ORC_THREADS).hex()
    assert got[1] == oracle.stream_blake3_mt(57, 11, L - 4096 - 5, ORC_THREADS).hex()
    del arena
    torch.cuda.empty_cache()


def test_file_checksums_many_paths(eng, oracle, tmp_path):
    """The validator job over a directory (sd_cas_file_checksums): small and empty files,
    files straddling the window and the streaming threshold, a missing path, a procfs file
    with st_size 0 (read to EOF), vs the oracle's file_checksum per path."""
    rng = np.random.default_rng(10)
    sizes = ([0, 1, 1023, 1024, 1025, (1 << 20) + 3, (64 << 20) + 1, (70 << 20) + 5]
             + [int(x) for x in rng.integers(0, 2 << 20, 120)] + [int(x) for x in rng.integers(20 << 20, 40 << 20, 8)])
    paths = []
    for i, L in enumerate(sizes):
        p = tmp_path / f"c{i}"
        p.write_bytes(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        paths.append(str(p))
    paths.insert(5, str(tmp_path / "missing"))
    # st_size 0 with content: /proc/sys/kernel/ostype fits its 128-B slot; /proc/filesystems
    # (a few hundred static bytes) overflows it, which sends the file through the streaming
    # redo path
    for proc in ("/proc/sys/kernel/ostype", "/proc/filesystems"):
        if os.path.exists(proc) and os.stat(proc).st_size == 0:
            paths.append(proc)
    digests, errs = eng.file_checksums(paths)
    for p, d, e in zip(paths, digests, errs):
        if p.endswith("missing"):
            assert d is None and e == 2
            continue
        assert e == 0 and d == oracle.file_checksum(p), p
    d0, e0 = eng.file_checksums([])
    assert d0 == [] and len(e0) == 0


def test_file_checksums_many_small_files(eng, oracle, tmp_path):
    """More files than one gather window holds (32,768): 40,000 files of 0-2 KiB, split over
    windows by file count, every digest vs the oracle."""
    d = "/dev/shm" if os.path.isdir("/dev/shm") else str(tmp_path)
    root = os.path.join(d, f"sdcas_many_{os.getpid()}")
    os.makedirs(root)
    rng = np.random.default_rng(12)
    paths = []
    try:
        for i, L in enumerate(rng.integers(0, 2049, 40_000)):
            p = os.path.join(root, f"{i}")
            with open(p, "wb") as fh:
                fh.write(rng.integers(0, 256, int(L), dtype=np.uint8).tobytes())
            paths.append(p)
        digests, errs = eng.file_checksums(paths)
        assert not errs.any()
        bad = [p for p, g in zip(paths, digests) if g != oracle.file_checksum(p)]
        assert not bad, bad[:3]
    finally:
        for p in paths:
            os.unlink(p)
        os.rmdir(root)


def test_file_checksums_pieces_and_slot_rotation(eng, oracle):
    """Round 6 piece queue of sd_cas_file_checksums: files read as 1 MiB pieces (the last piece
    takes the rest, incl. the EOF probe byte), lengths at every piece-count boundary, ~700 MB
    so the windows rotate over the three pinned slots twice, missing paths between, and the
    same files again (a second call reuses the grown staging) — every digest vs the oracle."""
    d = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
    root = os.path.join(d, f"sdcas_pieces_{os.getpid()}")
    os.makedirs(root)
    rng = np.random.default_rng(16)
    M = 1 << 20
    sizes = [k * M + e for k in (1, 2, 3) for e in (-129, -128, -127, -1, 0, 1, 127, 128)]
    sizes += [int(x) for x in rng.integers(M // 2, 3 * M, 400)]
    rng.shuffle(sizes)
    paths = []
    try:
        for i, L in enumerate(sizes):
            p = os.path.join(root, f"{i}")
            with open(p, "wb") as fh:
                fh.write(rng.integers(0, 256, int(L), dtype=np.uint8).tobytes())
            paths.append(p)
            if i % 97 == 5:
                paths.append(os.path.join(root, f"missing{i}"))
        assert sum(sizes) > 5 * (128 << 20)
        want = {p: oracle.file_checksum(p) for p in paths if "missing" not in p}
        for _ in range(2):
            digests, errs = eng.file_checksums(paths)
            for p, g, e in zip(paths, digests, errs):
                if "missing" in p:
                    assert g is None and e == 2
                else:
                    assert e == 0 and g == want[p], p
    finally:
        for p in paths:
            if os.path.exists(p):
                os.unlink(p)
        os.rmdir(root)


def test_file_checksums_big_files_one_queue(eng, oracle):
    """Round 6: regular files over 64 MiB go through ONE piece queue of 64 MiB segments (all
    files back to back), and sd_cas_file_checksum through the same queue for one file —
    sizes at segment multiples (a probe-only last segment), one byte either side, the empty
    file, small files between them (the windows), every digest vs the oracle; then the same
    big files one at a time through file_checksum."""
    d = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
    root = os.path.join(d, f"sdcas_big_{os.getpid()}")
    os.makedirs(root)
    rng = np.random.default_rng(19)
    M = 1 << 20
    sizes = [64 * M + 1, 5 * M, 128 * M, 0, 128 * M + 1, 3, 192 * M - 1, 65 * M, 64 * M]
    paths = []
    try:
        block = rng.integers(0, 256, 8 * M, dtype=np.uint8)
        for i, L in enumerate(sizes):
            p = os.path.join(root, f"b{i}")
            with open(p, "wb") as fh:
                left, k = L, 0
                while left:  # distinct bytes per file and per 8 MiB block
                    n = min(left, 8 * M)
                    fh.write((block[:n] ^ np.uint8((i * 31 + k) & 255)).tobytes())
                    left -= n
                    k += 1
            paths.append(p)
        want = [oracle.file_checksum(p) for p in paths]
        got, errs = eng.file_checksums(paths)
        assert not errs.any() and got == want
        for p, w in zip(paths, want):
            if os.path.getsize(p) >= 64 * M:
                assert eng.file_checksum(p) == w, p
    finally:
        for p in paths:
            os.unlink(p)
        os.rmdir(root)


def test_host_pool_numa_modes_agree(eng, oracle, monkeypatch, tmp_path):
    """Round 6: the host gather pool is bound to the GPU's NUMA node unless SD_CAS_POOL_NUMA=0
    (read at context creation).  A context of each mode gives the same validator digests and
    cas_ids for the same files (the sampled and whole-file gather, the piece queue), equal
    to the oracle."""
    from spacedrive_amd import CasEngine
    rng = np.random.default_rng(17)
    sizes = [0, 5, 1 << 20, (1 << 20) + 1, 3 << 20] + [int(x) for x in rng.integers(1, 400_000, 60)]
    paths = []
    for i, L in enumerate(sizes):
        p = tmp_path / f"n{i}"
        p.write_bytes(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        paths.append(str(p))
    want_sums = [oracle.file_checksum(p) for p in paths]
    got = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SD_CAS_POOL_NUMA", mode)
        e = CasEngine(0)
        sums, errs = e.file_checksums(paths)
        assert not errs.any() and sums == want_sums, mode
        keys, kerr = e.generate_cas_keys_from_paths(paths[1:], np.array(sizes[1:], dtype=np.int64))
        assert not kerr.any(), mode
        got[mode] = keys
    assert (got["1"] == got["0"]).all()
    assert [f"{k:016x}" for k in got["1"]] == [oracle.generate_cas_id(p, s) for p, s in zip(paths[1:], sizes[1:])]


def test_host_pool_private_fds(eng, oracle, monkeypatch, tmp_path):
    """Round 6: the pool's threads start on private descriptor tables (HostPool::
    set_private_fds, SD_CAS_POOL_PRIVATE_FDS; read at context creation) and keep only 0-2 and
    the HIP runtime's device descriptors of the copy.  Both modes give the oracle's digests and
    cas_ids — the validator's batch windows, its queue of files over 64 MiB, the single-file
    pieces mode (its readers open the file themselves) and the sampled / whole-file gather — and
    a pipe the caller closes after the pool started still reaches EOF (the copies are dropped)."""
    import os
    import select
    from spacedrive_amd import CasEngine
    rng = np.random.default_rng(23)
    sizes = [1, 4096, 100 * 1024, 100 * 1024 + 1, 3 << 20, (64 << 20) + 4097] + \
        [int(x) for x in rng.integers(1, 600_000, 40)]
    paths = []
    for i, L in enumerate(sizes):
        p = tmp_path / f"p{i}"
        p.write_bytes(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        paths.append(str(p))
    want_sums = [oracle.file_checksum(p) for p in paths]
    want_ids = [oracle.generate_cas_id(p, s) for p, s in zip(paths, sizes)]

    def tasks_without(fd):
        n = 0
        for t in os.listdir("/proc/self/task"):
            try:
                if str(fd) not in os.listdir(f"/proc/self/task/{t}/fd"):
                    n += 1
            except OSError:
                pass
        return n

    for mode in ("1", "0"):
        monkeypatch.setenv("SD_CAS_POOL_PRIVATE_FDS", mode)
        r, w = os.pipe()
        try:
            before = tasks_without(r)
            e = CasEngine(0)
            sums, errs = e.file_checksums(paths)
            assert not errs.any() and sums == want_sums, mode
            assert e.file_checksum(paths[4]) == want_sums[4], mode
            keys, kerr = e.generate_cas_keys_from_paths(paths, np.array(sizes, dtype=np.int64))
            assert not kerr.any(), mode
            assert [f"{k:016x}" for k in keys] == want_ids, mode
            keys100, _ = e.generate_cas_keys_from_paths(paths[:30], np.array(sizes[:30], dtype=np.int64))
            assert [f"{k:016x}" for k in keys100] == want_ids[:30], mode
            if mode == "1":  # the new pool's threads hold no copy of the caller's pipe
                assert tasks_without(r) > before
            os.close(w)
            w = -1
            ready, _, _ = select.select([r], [], [], 10.0)
            assert ready and os.read(r, 1) == b"", mode  # EOF: no thread holds the write end
            del e
        finally:
            os.close(r)
            if w >= 0:
                os.close(w)


def test_synth_matches_oracle_generator(eng, oracle):
    n, seed = 64, 12345
    content = torch.empty((n, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
    sizes = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_sampled(seed, 1000, n, content, sizes, SAMPLED_CONTENT_LEN, dup_permille=300)
    c = content.cpu().numpy()
    s = host64(sizes)
    roots = set()
    for i in range(n):
        root = oracle.synth_root(seed, 1000 + i, 300)
        roots.add(root)
        assert c[i].tobytes() == oracle.fill_content(seed, root, SAMPLED_CONTENT_LEN)
        assert int(s[i]) == oracle.synth_size(seed, root, 0)
    assert len(roots) < n  # the 30 % duplicate chain is exercised


def test_bench_scale_properties(eng, oracle):
    """At bench scale (1.25M sampled files/GPU, 72 GB in HBM): parity on a random subset and
    grouping == the generator's duplicate truth for every file."""
    n, seed, dup = 1_250_000, 77, 300
    content = torch.empty((n, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
    sizes = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_sampled(seed, 0, n, content, sizes, SAMPLED_CONTENT_LEN, dup_permille=dup)
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.hash_sampled(content, sizes, keys)
    rep = torch.empty(n, dtype=torch.int32, device="cuda")
    objects = eng.group(keys, rep)
    roots = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_roots(seed, 0, n, roots, dup_permille=dup)
    r = roots.cpu().numpy()
    uniq, inv = np.unique(r, return_inverse=True)
    first = np.full(len(uniq), n, dtype=np.int64)
    np.minimum.at(first, inv, np.arange(n))
    assert objects == len(uniq)
    assert (rep.cpu().numpy() == first[inv]).all()
    idx = np.random.default_rng(9).choice(n, 3000, replace=False)
    sub = content[torch.from_numpy(idx).cuda()].cpu().numpy()
    want = oracle.fast_cas_keys_strided(sub.reshape(-1), SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN,
                                        host64(sizes)[idx], 8)
    assert (host64(keys)[idx] == want).all()
    del content


def test_sampled_quantum_plus_remainder(eng, oracle):
    """Default dispatch of a batch that is not a whole number of quanta: K1 over the whole
    quanta, then K1L (either shape) on the remainder — identical keys to K1 on everything,
    and to the oracle across the boundary."""
    q = eng.batch_quantum
    for r in (1000, 5000):  # remainder on the wave-per-file / four-per-wave K1L shape
        n = q + r
        content = torch.empty((n, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
        sizes = torch.empty(n, dtype=torch.int64, device="cuda")
        eng.synth_sampled(31 + r, 0, n, content, sizes, SAMPLED_CONTENT_LEN)
        auto = torch.empty(n, dtype=torch.int64, device="cuda")
        eng.hash_sampled(content, sizes, auto)
        eng.set_latency_threshold(0, 0)
        lane = torch.empty(n, dtype=torch.int64, device="cuda")
        eng.hash_sampled(content, sizes, lane)
        eng.set_latency_threshold()
        assert torch.equal(auto, lane), r
        idx = np.arange(q - 300, q + 300)
        sub = content[q - 300:q + 300].cpu().numpy()
        want = oracle.fast_cas_keys_strided(sub.reshape(-1), SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN,
                                            host64(sizes)[idx], 8)
        assert (host64(auto)[idx] == want).all(), r
        del content


def test_k1_grids_agree(eng, oracle):
    """K1's two grid shapes (512-lane workgroups for an even number of quanta, 256-lane
    otherwise) give the same keys: 3 quanta (narrow grid) vs their first 2 quanta (wide
    grid) vs the first quantum and a 1.5-quantum batch (narrow K1 + K1L remainder), with
    oracle parity on 1,500 random files."""
    q = eng.batch_quantum
    n = 3 * q
    content = torch.empty((n, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
    sizes = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_sampled(0x6D1, 0, n, content, sizes, SAMPLED_CONTENT_LEN, dup_permille=100)
    runs = {}
    for m in (n, 2 * q, q, q + q // 2):
        k = torch.empty(m, dtype=torch.int64, device="cuda")
        eng.hash_sampled(content, sizes, k, n=m)
        runs[m] = host64(k)
    for m, k in runs.items():
        assert (k == runs[n][:m]).all(), m
    rng = np.random.default_rng(90)
    idx = np.sort(rng.choice(n, 1500, replace=False))
    sub = content[torch.from_numpy(idx).cuda()].cpu().numpy()
    want = oracle.fast_cas_keys_strided(sub.reshape(-1), SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN,
                                        host64(sizes)[idx], 8)
    assert (runs[n][idx] == want).all()


def test_config1_10k_files_tmpfs(eng, oracle):
    """BASELINE config 1 at its stated size: 10k files, sizes log-uniform in
    1 KiB..10 MiB (~11 GB) on /dev/shm, seeded as tools/bench_configs.py does, through
    sd_cas_generate_cas_ids_from_paths (the pread gather at the cas.rs:27-58 offsets) — every
    cas_id vs the oracle's literal read/seek generate_cas_id (cas.rs:23-62) — then the whole
    job through identifier_job_step (library-taken metadata, link emission) vs the replay."""
    import math
    import shutil

    import spacedrive_amd as sd
    rng = np.random.default_rng(1)
    n = 10_000
    sizes = np.exp(rng.uniform(math.log(1024), math.log(10 * 1024 * 1024), n)).astype(np.int64)
    root = f"/dev/shm/sdcas_cfg1_{os.getpid()}"
    os.makedirs(root, exist_ok=True)
    try:
        paths = []
        for i, s in enumerate(sizes):
            p = os.path.join(root, f"f{i:05d}")
            with open(p, "wb") as fh:
                fh.write(rng.integers(0, 256, int(s), dtype=np.uint8).tobytes())
            paths.append(p)
        keys, status = eng.generate_cas_keys_from_paths(paths, sizes)
        assert not status.any()
        want = [int(oracle.generate_cas_id(p, int(s)), 16) for p, s in zip(paths, sizes)]
        assert (keys == np.array(want, dtype=np.uint64)).all()
        res = sd.identifier_job_step(paths, eng=eng)
        step, obj, act, counts = replay_identifier_job(want, [0] * n, 100)
        assert [(b.total_created, b.total_linked) for b in res.steps] == counts
        assert res.object_of == {i: o for i, o in enumerate(obj)}
        assert all(res.metadata[i].size == int(sizes[i]) for i in range(n))
    finally:
        shutil.rmtree(root, ignore_errors=True)


def test_config2_1m_whole_files(eng, oracle):
    """BASELINE config 2 at its stated size: 1M whole-file messages (sizes
    uniform in 1..102,400, ~51 GB, seed as tools/bench_configs.py) resident in HBM through
    K2 — EVERY key vs the oracle's 16-thread AVX-512 restatement (oracle/cas_fast.c)."""
    n = 1_000_000
    sz = torch.empty(n, dtype=torch.int64, device="cuda")
    ln = torch.empty(n, dtype=torch.int32, device="cuda")
    of = torch.empty(n, dtype=torch.int64, device="cuda")
    nb = eng.synth_small(11, 0, n, sz, ln, of, None)
    arena = torch.empty(nb + 64, dtype=torch.uint8, device="cuda")
    eng.synth_small(11, 0, n, sz, ln, of, arena)
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.hash_packed(arena, of, ln, sz, keys)
    lens = ln.cpu().numpy().astype(np.uint64)
    assert lens.min() <= 1024 and lens.max() >= 100_000 and nb > 45e9
    host = arena.cpu().numpy()
    del arena
    torch.cuda.empty_cache()
    want = oracle.fast_cas_keys(host, of.cpu().numpy().astype(np.uint64), lens, host64(sz), 16)
    assert (host64(keys) == want).all()


def test_random_cases_1e5(path_eng, oracle):
    """SURVEY §7's minimum-slice bar on every kernel shape: 10^5 random whole-file messages
    (sizes uniform in [0, 102,400]) and 10^5 random sampled files, every cas key vs the
    oracle's SIMD restatement."""
    eng = path_eng
    n = 100_000
    sz = torch.empty(n, dtype=torch.int64, device="cuda")
    ln = torch.empty(n, dtype=torch.int32, device="cuda")
    of = torch.empty(n, dtype=torch.int64, device="cuda")
    nb = eng.synth_small(77, 0, n, sz, ln, of, None)
    arena = torch.empty(nb + 64, dtype=torch.uint8, device="cuda")
    eng.synth_small(77, 0, n, sz, ln, of, arena)
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.hash_packed(arena, of, ln, sz, keys)
    lens = ln.cpu().numpy().astype(np.uint32)
    assert lens.min() < 1024 and lens.max() > 100_000  # the whole 1 B .. 100 KiB range
    want = oracle.fast_cas_keys(arena.cpu().numpy(), of.cpu().numpy().astype(np.uint64), lens,
                                host64(sz), 8)
    assert (host64(keys) == want).all()
    del arena
    content = torch.empty((n, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
    sizes = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_sampled(78, 0, n, content, sizes, SAMPLED_CONTENT_LEN)
    eng.hash_sampled(content, sizes, keys)
    want = oracle.fast_cas_keys_strided(content.cpu().numpy().reshape(-1), SAMPLED_CONTENT_LEN,
                                        SAMPLED_CONTENT_LEN, host64(sizes), 8)
    assert (host64(keys) == want).all()
    del content


def test_headline_10m_files(eng, oracle):
    """BASELINE's target at its full size: 10M sampled files with 30 % duplicate content,
    hashed in 8 resident batches of 1.25M (71.7 GB each), cas_ids bit-exact vs the oracle on
    400 random files of every batch, and the Object grouping of all 10M keys == the
    generator's duplicate truth for every file — locally (K4h/K5h) and through the 8-way
    key-range exchange of the multi-GPU path (8 shards on this device, sd_cas_multi_group)."""
    from spacedrive_amd.multi import MultiEngine
    n, batch, seed, dup = 10_000_000, 1_250_000, 0x5DCA50004, 300
    content = torch.empty((batch, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
    sizes = torch.empty(batch, dtype=torch.int64, device="cuda")
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    rng = np.random.default_rng(100)
    for f0 in range(0, n, batch):
        eng.synth_sampled(seed, f0, batch, content, sizes, SAMPLED_CONTENT_LEN, dup_permille=dup)
        eng.hash_sampled(content, sizes, keys[f0:f0 + batch])
        idx = np.sort(rng.choice(batch, 400, replace=False))
        sub = content[torch.from_numpy(idx).cuda()].cpu().numpy()
        want = oracle.fast_cas_keys_strided(sub.reshape(-1), SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN,
                                            host64(sizes)[idx], 8)
        assert (host64(keys[f0:f0 + batch])[idx] == want).all(), f0
    del content
    roots = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_roots(seed, 0, n, roots, dup_permille=dup)
    r = roots.cpu().numpy()
    del roots
    uniq, inv = np.unique(r, return_inverse=True)
    first = np.full(len(uniq), n, dtype=np.int64)
    np.minimum.at(first, inv, np.arange(n))
    truth = first[inv]
    rep = torch.empty(n, dtype=torch.int32, device="cuda")
    objects = eng.group(keys, rep)
    assert objects == len(uniq)
    assert (rep.cpu().numpy() == truth).all()
    me = MultiEngine([0] * 8)
    cuts = [n * i // 8 for i in range(9)]
    reps, mobjects = me.group([keys[cuts[i]:cuts[i + 1]] for i in range(8)], cuts[:-1])
    assert mobjects == len(uniq)
    assert (np.concatenate([x.cpu().numpy() for x in reps]) == truth).all()
    me.close()


def test_config4_100m_files(eng, oracle):
    """BASELINE config 4 at its full size on one GPU: 100M sampled files with 30 % duplicate
    content, hashed in 80 resident batches of 1.25M (content regenerated on the device per
    batch), cas keys bit-exact vs the oracle on 200 random files of every batch, then the
    Object grouping of ALL 100M keys in one call (hash partition plan b1 = 8, b2 = 8) ==
    the generator's duplicate truth for every file — locally and through the 8-shard
    key-range exchange of the multi-GPU path (sd_cas_multi_group, 8 shards on this device).
    Truth: file f's content is that of synth_root(f), the first file of its duplicate
    chain, so the canonical representative of f is exactly its root."""
    import time as _t

    from spacedrive_amd.multi import MultiEngine
    n, batch, seed, dup = 100_000_000, 1_250_000, 0x5DCA50004 + 4, 300
    content = torch.empty((batch, SAMPLED_CONTENT_LEN), dtype=torch.uint8, device="cuda")
    sizes = torch.empty(batch, dtype=torch.int64, device="cuda")
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    rng = np.random.default_rng(101)
    t0 = _t.time()
    for f0 in range(0, n, batch):
        eng.synth_sampled(seed, f0, batch, content, sizes, SAMPLED_CONTENT_LEN, dup_permille=dup)
        eng.hash_sampled(content, sizes, keys[f0:f0 + batch])
        idx = np.sort(rng.choice(batch, 200, replace=False))
        sub = content[torch.from_numpy(idx).cuda()].cpu().numpy()
        want = oracle.fast_cas_keys_strided(sub.reshape(-1), SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN,
                                            host64(sizes)[idx], 8)
        assert (host64(keys[f0:f0 + batch])[idx] == want).all(), f0
        if f0 % (20 * batch) == 0:
            print(f"  hashed {f0 + batch:,} files, {_t.time() - t0:.1f}s", flush=True)
    del content
    torch.cuda.empty_cache()
    roots = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_roots(seed, 0, n, roots, dup_permille=dup)
    truth = roots.cpu().numpy()
    del roots
    n_obj = int(np.count_nonzero(truth == np.arange(n, dtype=np.int64)))
    rep = torch.empty(n, dtype=torch.int32, device="cuda")
    objects = eng.group(keys, rep)
    assert objects == n_obj
    assert (rep.cpu().numpy() == truth).all()
    del rep
    print(f"  grouped 100M keys locally: {objects:,} Objects, {_t.time() - t0:.1f}s", flush=True)
    me = MultiEngine([0] * 8)
    cuts = [n * i // 8 for i in range(9)]
    reps, mobjects = me.group([keys[cuts[i]:cuts[i + 1]] for i in range(8)], cuts[:-1])
    assert mobjects == n_obj
    for i in range(8):
        assert (reps[i].cpu().numpy() == truth[cuts[i]:cuts[i + 1]]).all(), i
    del reps
    me.close()


def test_identifier_job_step(eng, oracle, tmp_path):
    import spacedrive_amd as sd
    rng = np.random.default_rng(10)
    blobs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes()
             for s in [10, 5000, 102400, 150_000, 900_000]]
    paths = []
    for i in range(260):
        p = tmp_path / f"p{i:03d}"
        if i % 37 == 5:
            p.write_bytes(b"")  # empty: no cas_id, own Object (mod.rs:78-86)
        else:
            p.write_bytes(blobs[int(rng.integers(0, len(blobs)))] if rng.random() < 0.5
                          else rng.integers(0, 256, int(rng.integers(1, 200_000)), dtype=np.uint8).tobytes())
        paths.append(str(p))
    # an empty file at a chunk's last row (re-queried by the next step) and a missing one
    open(paths[198], "wb").close()
    os.unlink(paths[99])
    res = sd.identifier_job_step(paths, eng=eng)
    keys, states = [], []
    for p in paths:
        if not os.path.exists(p):
            keys.append(0); states.append(2)
            continue
        size = os.path.getsize(p)
        keys.append(0 if size == 0 else int(oracle.generate_cas_id(p, size), 16))
        states.append(1 if size == 0 else 0)
    assert res.errors == {99: 2}
    for i in range(len(paths)):
        if i in res.errors:
            continue
        want = None if states[i] else f"{keys[i]:016x}"
        assert res.metadata[i].cas_id == want
    step, obj, act, counts, creates = replay_identifier_job(keys, states, 100, with_creates=True)
    assert {i: o for i, (o, a) in enumerate(zip(obj, act)) if a in (0, 1)} == res.object_of
    assert [(b.total_created, b.total_linked) for b in res.steps] == counts
    assert (res.total_created, res.total_linked) == tuple(map(sum, zip(*counts)))
    # every step's create batch, including the empty row 198 that ends step 1's chunk and is
    # created again by step 2 (creates.len() == total_created per step)
    assert [b.creates for b in res.steps] == creates
    assert 198 in res.steps[1].creates and 198 in res.steps[2].creates
    for b in res.steps:
        assert len(b.creates) == b.total_created
        assert all(act[r] == 0 for r in b.creates)
        assert all(step[r] == b.step and obj[r] == o and act[r] == 1 for r, o in b.links)


@pytest.mark.parametrize("chunk", [100, 7, 2, 1])
def test_identifier_links_vs_replay(eng, chunk):
    """sd_cas_identifier_links_dev vs the literal DB replay of a whole job
    (file_identifier_job.rs:180-236, mod.rs:98-350) with the reference's cursor: rows that
    stay orphan (errors, empty files) at a chunk's last row are queried again by the next
    step (mod.rs:401-405, file_identifier_job.rs:268), the job stops after ceil(n/chunk)
    steps, duplicates inside and across steps, and error/empty runs at the table's end."""
    rng = np.random.default_rng(80 + chunk)
    n = 20_000 if chunk > 2 else 3_000
    pool = rng.integers(1, 2 ** 64, n // 3, dtype=np.uint64)
    keys = pool[rng.integers(0, len(pool), n)]
    states = rng.choice(np.array([0, 1, 2], dtype=np.uint8), n, p=[0.9, 0.05, 0.05])
    last_rows = np.arange(chunk - 1, n, chunk)  # chunk ends: many stay-orphan rows
    states[last_rows[rng.random(len(last_rows)) < 0.3]] = 2
    states[last_rows[rng.random(len(last_rows)) < 0.2]] = 1
    states[-5:] = [0, 1, 2, 1, 2]
    want_step, want_obj, want_act, want_counts = replay_identifier_job(
        [int(k) for k in keys], [int(s) for s in states], chunk)
    step, obj, act, counts = eng.identifier_links(dev64(keys), torch.from_numpy(states).cuda(), chunk)
    assert [tuple(c) for c in counts.tolist()] == want_counts
    assert (step.cpu().numpy().view(np.uint32) == np.array(want_step, dtype=np.uint32)).all()
    assert (obj.cpu().numpy().view(np.uint32) == np.array(want_obj, dtype=np.uint32)).all()
    assert (act.cpu().numpy() == np.array(want_act, dtype=np.uint8)).all()


@pytest.mark.parametrize("chunk", [100, 7, 1])
def test_identifier_links_existing_vs_replay(eng, chunk):
    """sd_cas_identifier_links_seeded[_dev] vs the replay on a library that already holds
    Objects (mod.rs:180-253): ~30 % of the keys carry pre-job Objects (some
    several, ids in any order), existing keys repeat inside one chunk, NO_CAS/ERROR rows end
    chunks, and a seed key no row has.  Device and host entry points, with and without
    per-row states."""
    rng = np.random.default_rng(180 + chunk)
    n = 12_000 if chunk > 2 else 2_500
    pool = rng.integers(1, 2 ** 64, n // 4, dtype=np.uint64)
    keys = pool[rng.integers(0, len(pool), n)]
    keys[10:14] = keys[10]  # one existing-or-fresh key four times inside one chunk
    states = rng.choice(np.array([0, 1, 2], dtype=np.uint8), n, p=[0.9, 0.05, 0.05])
    last_rows = np.arange(chunk - 1, n, chunk)
    states[last_rows[rng.random(len(last_rows)) < 0.3]] = 2
    states[last_rows[rng.random(len(last_rows)) < 0.2]] = 1
    if chunk == 1:  # every row ends its chunk: a row that stays orphan is re-queried until
        states[:] = 0  # the step budget runs out (the reference's cursor), so only at the end
        states[-3:] = [1, 0, 2]
    pre = pool[rng.random(len(pool)) < 0.3]
    pre = np.concatenate([pre, [keys[10], np.uint64(12345)]]).astype(np.uint64)
    ids = rng.permutation(3 * len(pre))[:len(pre)].astype(np.uint32)      # unordered ids
    extra = rng.integers(0, len(pre), len(pre) // 5)                      # several per key
    sk = np.concatenate([pre, pre[extra]])
    so = np.concatenate([ids, rng.integers(0, 2 ** 31 - 1, len(extra)).astype(np.uint32)])
    existing = list(zip((int(k) for k in sk), (int(o) for o in so)))
    for st in (states, None):
        want_step, want_obj, want_act, want_counts = replay_identifier_job(
            [int(k) for k in keys], [int(s) for s in (st if st is not None else np.zeros(n))], chunk,
            existing=existing)
        assert 4 in want_act and 0 in want_act and 1 in want_act
        step, obj, act, counts = eng.identifier_links(
            dev64(keys), None if st is None else torch.from_numpy(st).cuda(), chunk,
            existing=(dev64(sk), torch.from_numpy(so.view(np.int32)).cuda()))
        assert [tuple(c) for c in counts.tolist()] == want_counts
        assert (step.cpu().numpy().view(np.uint32) == np.array(want_step, dtype=np.uint32)).all()
        assert (obj.cpu().numpy().view(np.uint32) == np.array(want_obj, dtype=np.uint32)).all()
        assert (act.cpu().numpy() == np.array(want_act, dtype=np.uint8)).all()
        hstep, hobj, hact, hcounts = eng.identifier_links_host(keys, st, chunk, existing=(sk, so))
        assert [tuple(c) for c in hcounts.tolist()] == want_counts
        assert (hobj == np.array(want_obj, dtype=np.uint32)).all()
        assert (hact == np.array(want_act, dtype=np.uint8)).all()
    # an empty seed is the fresh-library call; an id >= 2^31 is refused
    a = eng.identifier_links_host(keys, states, chunk, existing=(sk[:0], so[:0]))
    b = eng.identifier_links_host(keys, states, chunk)
    assert all((x == y).all() for x, y in zip(a, b))
    from spacedrive_amd import CasError
    with pytest.raises(ValueError):  # the Python wrapper refuses it before the call ...
        eng.identifier_links_host(keys, states, chunk, existing=(sk[:1], np.array([2 ** 31], np.uint32)))
    # ... the device entry point checks the ids on the device (an id >= 2^31 would
    # read as a row tag), a negative int32 included
    with pytest.raises(CasError):
        eng.identifier_links(dev64(keys), torch.from_numpy(states).cuda(), chunk,
                             existing=(dev64(sk[:2]), torch.tensor([5, -7], dtype=torch.int32).cuda()))


@pytest.mark.parametrize("chunk", [100, 7, 1])
def test_identifier_links_pre_objects_vs_replay(eng, chunk):
    """sd_cas_identifier_links_ex[_dev] vs the literal replay with rows that ALREADY OWN an
    Object (object_id set, cas_id NULL: orphan by file_identifier_job.rs:258-261; VERDICT r4
    #1): ~10 % of rows carry a pre-existing Object, a key with one repeats inside its chunk
    and across chunks (a pre-job Object taking over a key an earlier step created), combined
    with seeded Objects (ids interleaved), NO_CAS / ERROR rows with Objects, stay-orphan rows
    at chunk ends.  Device and host entry points; an id >= 2^31 is refused on both."""
    rng = np.random.default_rng(280 + chunk)
    n = 12_000 if chunk > 2 else 2_500
    pool = rng.integers(1, 2 ** 64, n // 4, dtype=np.uint64)
    keys = pool[rng.integers(0, len(pool), n)]
    keys[20:26] = keys[20]           # one key six times inside one chunk, with an Object at 23
    keys[[150, 420, 900]] = keys[20]  # ... and in later chunks
    states = rng.choice(np.array([0, 1, 2], dtype=np.uint8), n, p=[0.9, 0.05, 0.05])
    last_rows = np.arange(chunk - 1, n, chunk)
    states[last_rows[rng.random(len(last_rows)) < 0.3]] = 2
    states[last_rows[rng.random(len(last_rows)) < 0.2]] = 1
    if chunk == 1:
        states[:] = 0
        states[-3:] = [1, 0, 2]
    states[20:26] = 0
    ids = rng.permutation(4 * n).astype(np.uint32)
    pre = np.where(rng.random(n) < 0.1, ids[:n], 0xFFFFFFFF).astype(np.uint32)
    pre[23] = 5
    pre[420] = 3  # smaller: takes the key over from row 23's Object in a later chunk
    seeded_keys = pool[rng.random(len(pool)) < 0.2]
    sk = seeded_keys.astype(np.uint64)
    so = ids[n:n + len(sk)].astype(np.uint32)
    pre_list = [None if int(p) == 0xFFFFFFFF else int(p) for p in pre]
    for existing in ((sk, so), None):
        ex = None if existing is None else list(zip((int(k) for k in sk), (int(o) for o in so)))
        want_step, want_obj, want_act, want_counts = replay_identifier_job(
            [int(k) for k in keys], [int(s) for s in states], chunk, existing=ex, pre_objects=pre_list)
        assert 4 in want_act and 0 in want_act
        step, obj, act, counts = eng.identifier_links(
            dev64(keys), torch.from_numpy(states).cuda(), chunk,
            existing=None if existing is None else (dev64(sk), torch.from_numpy(so.view(np.int32)).cuda()),
            pre_objects=torch.from_numpy(pre.view(np.int32)).cuda())
        assert [tuple(c) for c in counts.tolist()] == want_counts
        assert (step.cpu().numpy().view(np.uint32) == np.array(want_step, dtype=np.uint32)).all()
        assert (obj.cpu().numpy().view(np.uint32) == np.array(want_obj, dtype=np.uint32)).all()
        assert (act.cpu().numpy() == np.array(want_act, dtype=np.uint8)).all()
        hstep, hobj, hact, hcounts = eng.identifier_links_host(keys, states, chunk, existing=existing,
                                                               pre_objects=pre_list)
        assert [tuple(c) for c in hcounts.tolist()] == want_counts
        assert (hobj == np.array(want_obj, dtype=np.uint32)).all()
        assert (hact == np.array(want_act, dtype=np.uint8)).all()
    if chunk == 100:
        assert want_act[23] == 4 and want_obj[23] == 5 and want_obj[420] == 3 and want_obj[900] == 3
    # no row owning an Object = the seeded / fresh call
    none = np.full(n, 0xFFFFFFFF, np.uint32)
    a = eng.identifier_links_host(keys, states, chunk, existing=(sk, so), pre_objects=none)
    b = eng.identifier_links_host(keys, states, chunk, existing=(sk, so))
    assert all((x == y).all() for x, y in zip(a, b))
    from spacedrive_amd import CasError
    bad = pre.copy()
    bad[7] = 2 ** 31
    with pytest.raises(ValueError):
        eng.identifier_links_host(keys, states, chunk, pre_objects=bad)
    with pytest.raises(CasError):
        eng.identifier_links(dev64(keys), torch.from_numpy(states).cuda(), chunk,
                             pre_objects=torch.from_numpy(bad.view(np.int32)).cuda())


def test_identifier_links_pre_objects_edges(eng):
    """Edge shapes of sd_cas_identifier_links_ex against the replay: no rows; one row owning
    an Object; every row owning the same Object; Objects only on ERROR / NO_CAS rows (no
    event: the fresh answer); Objects on rows past the job's last step (not reached, so not
    seen); an Object id of 0 and of 2^31 - 1; chunk larger than the job."""
    from spacedrive_amd import NO_OBJECT  # noqa: F401  (re-exported constant)
    cases = []
    k = np.array([5, 5, 7, 5, 9, 7, 5], np.uint64)
    cases.append((k, np.zeros(7, np.uint8), [None, None, None, 0, None, 2 ** 31 - 1, None], 3, None))
    cases.append((k[:1], np.zeros(1, np.uint8), [42], 100, None))
    cases.append((k, np.zeros(7, np.uint8), [11] * 7, 2, None))
    st = np.array([2, 1, 0, 2, 1, 0, 0], np.uint8)
    cases.append((k, st, [3, 4, None, 5, 6, None, None], 3, None))
    # chunk 1 with a stay-orphan row in front: the job re-queries it until its steps run out,
    # so the later rows (with Objects) are never reached
    cases.append((k, np.array([2, 0, 0, 0, 0, 0, 0], np.uint8), [None, 8, 9, 1, 2, 3, 4], 1, None))
    cases.append((k, np.zeros(7, np.uint8), [None, 50, None, None, 40, None, 30], 2,
                  [(5, 60), (9, 35), (7, 70)]))
    for keys, states, pre, chunk, seeds in cases:
        want_step, want_obj, want_act, want_counts = replay_identifier_job(
            [int(x) for x in keys], [int(x) for x in states], chunk, existing=seeds, pre_objects=pre)
        po = np.array([0xFFFFFFFF if p is None else p for p in pre], np.uint32)
        ex = None
        if seeds:
            ex = (np.array([a for a, _ in seeds], np.uint64), np.array([b for _, b in seeds], np.uint32))
        step, obj, act, counts = eng.identifier_links(
            dev64(keys), torch.from_numpy(states).cuda(), chunk,
            existing=None if ex is None else (dev64(ex[0]), torch.from_numpy(ex[1].view(np.int32)).cuda()),
            pre_objects=torch.from_numpy(po.view(np.int32)).cuda())
        assert [tuple(c) for c in counts.tolist()] == want_counts, (pre, chunk)
        assert (step.cpu().numpy().view(np.uint32) == np.array(want_step, np.uint32)).all()
        assert (obj.cpu().numpy().view(np.uint32) == np.array(want_obj, np.uint32)).all(), (pre, chunk)
        assert (act.cpu().numpy() == np.array(want_act, np.uint8)).all(), (pre, chunk)
    # no rows at all
    e = torch.empty(0, dtype=torch.int64, device="cuda")
    step, obj, act, counts = eng.identifier_links(e, None, 100,
                                                  pre_objects=torch.empty(0, dtype=torch.int32, device="cuda"))
    assert step.numel() == 0 and counts.shape == (0, 2)


def test_identifier_links_job_at_library_scale(eng):
    """One identifier job over 50 M rows (half of config 4's 100 M-file library as ONE job):
    30 % duplicate keys, 2 % NO_CAS / ERROR rows (some at chunk ends: the cursor re-queries
    them), 5 % of rows owning an Object, seeds for 1 % of keys; chunk 100 (500 k steps) — every
    row's step, decision and owner vs the vectorised closed form of the replay
    (tests/golden/make_golden.py::closed_form, pinned against the replay by a CPU test)."""
    from tests.golden.make_golden import closed_form, cursor_walk
    rng = np.random.default_rng(505)
    n, chunk = 50_000_000, 100
    uniq = rng.integers(1, 2 ** 64, int(n * 0.7), dtype=np.uint64)
    keys = np.concatenate([uniq, uniq[rng.integers(0, len(uniq), n - len(uniq))]])
    rng.shuffle(keys)
    states = np.zeros(n, np.uint8)
    bad = rng.random(n) < 0.02
    states[bad] = rng.choice(np.array([1, 2], np.uint8), int(bad.sum()))
    pre = np.full(n, 0xFFFFFFFF, np.uint32)
    own = rng.random(n) < 0.05
    ids = rng.permutation(1 << 30)[: int(own.sum()) + len(uniq) // 100]
    pre[own] = ids[: int(own.sum())].astype(np.uint32)
    sk = uniq[: len(uniq) // 100]
    so = ids[int(own.sum()):int(own.sum()) + len(sk)].astype(np.uint32)
    step, obj, act, counts = eng.identifier_links(
        dev64(keys), torch.from_numpy(states).cuda(), chunk,
        existing=(dev64(sk), torch.from_numpy(so.view(np.int32)).cuda()),
        pre_objects=torch.from_numpy(pre.view(np.int32)).cuda())
    wstep, starts, _ = cursor_walk(states, n, chunk)
    assert (step.cpu().numpy().view(np.uint32).astype(np.int64) == wstep).all()
    wo, wa = closed_form(keys, states, pre, list(zip(sk.tolist(), so.tolist())), wstep, starts)
    assert (obj.cpu().numpy().view(np.uint32).astype(np.int64) == wo).all()
    assert (act.cpu().numpy().astype(np.int64) == wa).all()
    # per-step counts: every decided row once, plus a NO_CAS row a step re-queries (the
    # cursor's last row stays orphan) created again — at most one per step
    done = int(((wa == 0) | (wa == 1) | (wa == 4)).sum())
    total = int(counts[:, 0].sum()) + int(counts[:, 1].sum())
    assert done <= total <= done + len(starts) and len(counts) == len(starts)


def test_identifier_links_pre_objects_hot_key_1m(eng):
    """The two scans at scale: 1M rows, one hot key over every chunk with pre-existing
    Objects whose ids decrease step by step (each step's minimum takes over), plus random
    keys; every row hashed (chunk 100) vs the closed form of the replay."""
    rng = np.random.default_rng(281)
    n = 1 << 20
    keys = rng.integers(1, 2 ** 64, 700_000, dtype=np.uint64)[rng.integers(0, 700_000, n)]
    hot = np.arange(0, n, 37)
    keys[hot] = np.uint64(0xABCDEF)
    pre = np.full(n, 0xFFFFFFFF, np.uint32)
    owners = hot[::5]
    pre[owners] = (2 ** 30 - owners).astype(np.uint32)  # later rows, smaller ids
    some = rng.choice(n, n // 50, replace=False)
    pre[some] = rng.integers(0, 2 ** 31 - 1, len(some)).astype(np.uint32)
    step, obj, act, counts = eng.identifier_links(dev64(keys), None, 100,
                                                  pre_objects=torch.from_numpy(pre.view(np.int32)).cuda())
    st = np.arange(n) // 100
    assert (step.cpu().numpy() == st).all()
    # closed form: per key, the minimum pre-existing Object over rows in steps <= the row's
    order = np.lexsort((np.arange(n), keys))
    sk, sr = keys[order], order
    want = np.full(n, 0xFFFFFFFF, np.uint64)
    first = np.empty(n, np.int64)
    p = pre[sr].astype(np.uint64)
    starts = np.flatnonzero(np.r_[True, sk[1:] != sk[:-1]])
    for a, b in zip(starts, np.r_[starts[1:], n]):
        first[sr[a:b]] = sr[a]
        if b - a == 1:
            want[sr[a]] = p[a]
            continue
        pm = np.minimum.accumulate(p[a:b])
        s = st[sr[a:b]]
        last = np.r_[np.flatnonzero(s[1:] != s[:-1]), b - a - 1]   # end of each step's run
        want[sr[a:b]] = pm[last[np.searchsorted(last, np.arange(b - a))]]
    o = obj.cpu().numpy().view(np.uint32).astype(np.int64)
    a_ = act.cpu().numpy()
    ex = want != 0xFFFFFFFF
    assert (a_[ex] == 4).all() and (o[ex] == want[ex].astype(np.int64)).all()
    created = ~ex & (st[first] == st)
    assert (a_[created] == 0).all() and (o[created] == np.arange(n)[created]).all()
    linked = ~ex & ~created
    assert (a_[linked] == 1).all() and (o[linked] == first[linked]).all()
    assert ex[hot].sum() > len(hot) // 2 and linked.any() and created.any()
    # the hot key's target falls step by step: every owner row takes it over
    assert (o[owners] <= pre[owners]).all()
    assert int(counts[:, 0].sum()) + int(counts[:, 1].sum()) == n


def test_identifier_job_step_existing(eng, oracle, tmp_path):
    """identifier_job_step on a library whose earlier job already made Objects: the second
    location's files whose cas_id an older Object carries link to it (LINK_EXISTING), the
    others follow the fresh rules; FileMetadata.size is the metadata length the library used."""
    import spacedrive_amd as sd
    rng = np.random.default_rng(11)
    blobs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in [300, 150_000, 7]]
    paths = []
    for i in range(150):
        p = tmp_path / f"q{i:03d}"
        p.write_bytes(blobs[i % 3] if i % 4 == 0 else
                      rng.integers(0, 256, int(rng.integers(1, 130_000)), dtype=np.uint8).tobytes())
        paths.append(str(p))
    ids = {oracle.generate_cas_id(paths[0], os.path.getsize(paths[0])): 41,
           oracle.generate_cas_id(paths[4], os.path.getsize(paths[4])): 17}
    res = sd.identifier_job_step(paths, eng=eng, existing=(list(ids), list(ids.values())))
    for i, p in enumerate(paths):
        want = oracle.generate_cas_id(p, os.path.getsize(p))
        assert res.metadata[i].cas_id == want and res.metadata[i].size == os.path.getsize(p)
        if want in ids:
            assert res.existing_of[i] == ids[want] and i not in res.object_of
        else:
            assert i in res.object_of
    assert sum(len(b.links_existing) for b in res.steps) == len(res.existing_of) > 0
    assert res.total_linked == sum(len(b.links) + len(b.links_existing) for b in res.steps)


def test_identifier_job_step_watcher_sequence(eng, oracle, tmp_path):
    """The watcher's create-then-write sequence end to end: files created empty got an
    Object with no cas_id (watcher/utils.rs:236-293), then were written — the update keeps
    the old NULL cas_id with the new size (:473-490) — so the job's orphan query returns them
    with their Object (file_identifier_job.rs:258-261).  identifier_job_step(pre_objects=)
    hashes them and links them, and every file of their step with the same content, to the
    smallest such Object; one file still empty at identification time gets a new Object;
    decisions and per-step counts equal the literal replay on the oracle's cas_ids."""
    import spacedrive_amd as sd
    rng = np.random.default_rng(12)
    blobs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in [4_000, 180_000, 33]]
    paths, pre = [], []
    for i in range(230):
        p = tmp_path / f"w{i:03d}"
        p.write_bytes(b"")                       # the watcher's create: empty, Object made
        pre.append(1000 + 3 * i if i % 9 == 4 else None)
        paths.append(str(p))
    for i, p in enumerate(paths):                # ... then written
        if i == 121:
            continue                             # still empty: NO_CAS, a new Object
        open(p, "wb").write(blobs[i % 3] if i % 4 == 0 else
                            rng.integers(0, 256, int(rng.integers(1, 150_000)), dtype=np.uint8).tobytes())
    pre[121] = 7
    pre[8] = 2                                   # row 8 (blob 2) owns the smallest Object
    res = sd.identifier_job_step(paths, eng=eng, pre_objects=pre)
    keys = [0 if os.path.getsize(p) == 0 else int(oracle.generate_cas_id(p, os.path.getsize(p)), 16)
            for p in paths]
    states = [1 if k == 0 else 0 for k in keys]
    step, obj, act, counts = replay_identifier_job(keys, states, 100, pre_objects=pre)
    assert [(b.total_created, b.total_linked) for b in res.steps] == counts
    assert {i: o for i, (o, a) in enumerate(zip(obj, act)) if a == 4} == res.existing_of
    assert {i: o for i, (o, a) in enumerate(zip(obj, act)) if a in (0, 1)} == res.object_of
    assert res.existing_of[8] == 2 and 121 in res.object_of and res.object_of[121] == 121
    assert all(res.existing_of[i] == 2 for i in range(8, 100, 4) if i % 3 == 2)  # blob 2 in step 0
    assert res.metadata[4].cas_id == f"{keys[4]:016x}" and res.existing_of[4] <= 1000 + 12


def test_identifier_links_all_hashed_1m(eng, oracle):
    """Without per-row states (every row hashed, the device-resident re-identify batch) the
    emission equals the chunk replay (sd_cas_group_chunked_dev / the oracle) at 1M rows."""
    rng = np.random.default_rng(90)
    n = 1 << 20
    pool = rng.integers(0, 2 ** 64, 700_000, dtype=np.uint64)
    keys = pool[rng.integers(0, len(pool), n)]
    step, obj, act, counts = eng.identifier_links(dev64(keys), None, 100)
    crep, cc, cl = oracle.group_chunked(keys, 100)
    assert len(counts) == (n + 99) // 100
    assert (int(counts[:, 0].sum()), int(counts[:, 1].sum())) == (cc, cl)
    assert (obj.cpu().numpy().view(np.uint32) == crep).all()
    assert (step.cpu().numpy() == np.arange(n) // 100).all()
    a = act.cpu().numpy()
    assert ((a == 0) == (crep == np.arange(n, dtype=np.uint32))).all()


def test_sampled_host_pipeline(eng, oracle):
    """End-to-end path from (pinned) host memory: H2D of batch k+1 overlaps K1 on batch k."""
    rng = np.random.default_rng(12)
    n = 5000
    pinned = eng.alloc_pinned(n * SAMPLED_CONTENT_LEN)
    try:
        pinned[:] = rng.integers(0, 256, n * SAMPLED_CONTENT_LEN, dtype=np.uint8)
        sizes = rng.integers(MINIMUM_FILE_SIZE + 1, 2 ** 40, n, dtype=np.uint64)
        want = oracle.fast_cas_keys_strided(pinned, SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN, sizes, 8)
        for batch in [0, 1, 999, 1024, 5000]:
            got = eng.hash_sampled_host(pinned, sizes, batch_files=batch)
            assert (got == want).all(), batch
        # the ring form (bench e2e, config 3): 5,000 files cycling through the first 777 rows;
        # each batch's two halves cross on the two copy streams and wrap the ring mid-half
        ring = 777
        want_ring = want[:ring][np.arange(n) % ring]
        sizes_ring = sizes[:ring][np.arange(n) % ring]
        for batch in [1, 333, 1000, 4999]:
            got = eng.hash_sampled_host_ring(pinned.ctypes.data, ring, sizes_ring, batch_files=batch)
            assert (got == want_ring).all(), batch
    finally:
        eng.free_pinned(pinned)
    # pageable memory works too (synchronous copies)
    host = rng.integers(0, 256, 300 * SAMPLED_CONTENT_LEN, dtype=np.uint8)
    sizes = rng.integers(MINIMUM_FILE_SIZE + 1, 2 ** 40, 300, dtype=np.uint64)
    assert (eng.hash_sampled_host(host, sizes, batch_files=128) ==
            oracle.cas_keys_strided(host, SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN, sizes)).all()


def test_exchange_rows_vs_numpy(eng):
    """sd_cas_exchange_{pack,split,unpack}_dev: the 12-byte (key, u32 idx) rows of the RCCL
    exchange, with file0 near the top of the u32 range."""
    rng = np.random.default_rng(61)
    n = 100_003
    keys = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
    pos = rng.permutation(n).astype(np.int32)
    file0 = (1 << 32) - n
    rows = torch.empty((n, 3), dtype=torch.int32, device="cuda")
    eng.exchange_pack(dev64(keys), torch.from_numpy(pos).cuda(), file0, rows)
    r = rows.cpu().numpy().view(np.uint32)
    assert (r[:, 0] == (keys & 0xFFFFFFFF)).all() and (r[:, 1] == (keys >> np.uint64(32))).all()
    assert (r[:, 2] == pos.astype(np.uint64) + file0).all()
    k2 = torch.empty(n, dtype=torch.int64, device="cuda")
    v2 = torch.empty(n, dtype=torch.int32, device="cuda")
    eng.exchange_split(rows, k2, v2)
    assert (host64(k2) == keys).all() and (v2.cpu().numpy().view(np.uint32) == r[:, 2]).all()
    rep = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.exchange_unpack(v2, torch.from_numpy(pos).cuda(), rep)
    want = np.empty(n, dtype=np.int64)
    want[pos] = r[:, 2]
    assert (rep.cpu().numpy() == want).all()


def test_sharded_group_rccl_world1(eng, oracle):
    """The multi-GPU grouping path (spacedrive_amd/shard.py) on the GPU with the nccl (= RCCL)
    backend: world size 1 here (one GPU per box); the world-2/4 exchange logic is covered
    with gloo in tests/test_shard_cpu.py."""
    import socket

    import torch.distributed as dist

    from spacedrive_amd.shard import HipShardOps, sharded_group
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        rng = np.random.default_rng(13)
        pool = rng.integers(0, 2 ** 64, 40_000, dtype=np.uint64)
        keys = pool[rng.integers(0, len(pool), 100_000)]
        res = sharded_group(dev64(keys), 5_000_000, HipShardOps(eng))
        orep, oobj = oracle.group_canonical(keys)
        assert res.objects == oobj
        assert (res.rep.cpu().numpy() == orep.astype(np.int64) + 5_000_000).all()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_fixed_capacity_exchange_kernels(eng, oracle, world):
    """The HIP kernels of the sync-free exchange (sd_cas_exchange_{pack,split,unpack}_
    fixed_dev + sd_cas_copy_objects_dev) with `world` ranks emulated in one process: the
    all_to_all of equal blocks is a block transpose.  Grouping == the oracle's canonical,
    keys equal to the sentinels included; then an overflowing part sets the flag."""
    from spacedrive_amd.shard import HipShardOps, fixed_capacity, range_start
    ops = HipShardOps(eng)
    rng = np.random.default_rng(50 + world)
    pool = rng.integers(0, 2 ** 64, 60_000, dtype=np.uint64)
    for r in range(world):
        b = range_start(r, world)
        pool[2 * r: 2 * r + 2] = [b, (b - 1) % 2 ** 64]
    keys = pool[rng.integers(0, len(pool), 200_003)]
    cuts = [len(keys) * r // world for r in range(world + 1)]
    cap, spill = fixed_capacity(max(cuts[r + 1] - cuts[r] for r in range(world)), world)
    sent = []
    for r in range(world):
        k = dev64(keys[cuts[r]:cuts[r + 1]])
        pk, pp, cnt = ops.partition(k, world)
        rows, srows, ovf = ops.pack_fixed(pk, pp, cnt, world, cap, spill, cuts[r])
        sent.append((pp, cnt, rows.view(world, cap, 3), srows.view(world, spill, 3), ovf))
    assert all(int(s[4].item()) == 0 for s in sent)
    backs = []
    objects = 0
    for d in range(world):  # receiver d: block d of every sender, main then spill
        rr = torch.cat([s[2][d] for s in sent] + [s[3][d] for s in sent])
        rk, rv, nsent = ops.split_fixed(rr, range_start(d + 1, world))
        ku = rr[:, 0].cpu().numpy().view(np.uint32).astype(np.uint64) | (
            rr[:, 1].cpu().numpy().view(np.uint32).astype(np.uint64) << np.uint64(32))
        pad = ku == np.uint64(range_start(d + 1, world))
        assert int(nsent.item()) == int(pad.sum())
        got = rk.cpu().numpy().view(np.uint64)
        want = np.where(pad, np.uint64(range_start(d + 1, world)) + np.arange(len(ku), dtype=np.uint64), ku)
        assert (got == want).all()  # padding spread to distinct keys, real keys untouched
        out, obj = ops.group_min_dev(rk, rv)
        objects += int(obj.item()) - int(nsent.item())
        backs.append(out)
    orep, oobj = oracle.group_canonical(keys)
    assert objects == oobj
    for r in range(world):  # mirror: sender r gets block r of every receiver's reps
        back = torch.cat([b[:world * cap].view(world, cap)[r] for b in backs])
        sback = torch.cat([b[world * cap:].view(world, spill)[r] for b in backs])
        rep = ops.unpack_fixed(back, sback, sent[r][0], sent[r][1], world, cap, spill)
        assert (rep.cpu().numpy() == orep[cuts[r]:cuts[r + 1]].astype(np.int64)).all(), r
    # a part beyond cap + spill raises the overflow flag
    k = dev64(np.full(5000, keys[0], dtype=np.uint64))
    pk, pp, cnt = ops.partition(k, world)
    _, _, ovf = ops.pack_fixed(pk, pp, cnt, world, 100, 100, 0)
    assert int(ovf.item()) == 1


def test_multi_device_create_across_devices(eng, oracle):
    """sd_cas_multi_create over two distinct devices: on a one-GPU box it fails loudly
    (ENODEV, with the reason); with two or more GPUs peer access must be enabled and the
    cross-device exchange (hipMemcpyPeerAsync over xGMI) must match the oracle."""
    from spacedrive_amd import CasError
    from spacedrive_amd.multi import MultiEngine
    if torch.cuda.device_count() < 2:
        with pytest.raises(CasError, match="ENODEV.*device 1"):
            MultiEngine([0, 1])
        return
    rng = np.random.default_rng(24)
    pool = rng.integers(0, 2 ** 64, 40_000, dtype=np.uint64)
    keys = pool[rng.integers(0, len(pool), 100_000)]
    me = MultiEngine([0, 1])
    parts = [torch.from_numpy(keys[:50_000].view(np.int64)).to("cuda:0"),
             torch.from_numpy(keys[50_000:].view(np.int64)).to("cuda:1")]
    reps, objects = me.group(parts, [0, 50_000])
    orep, oobj = oracle.group_canonical(keys)
    assert objects == oobj
    assert (np.concatenate([r.cpu().numpy() for r in reps]) == orep.astype(np.int64)).all()
    me.close()


@pytest.mark.parametrize("shards", [1, 2, 3, 4])
def test_multi_device_group(eng, oracle, shards):
    """Single-process multi-device grouping (sd_cas_multi_group): `shards` shards on
    device 0, so the whole peer-copy exchange, split points and mirror run on one GPU."""
    from spacedrive_amd.multi import MultiEngine
    rng = np.random.default_rng(20 + shards)
    pool = rng.integers(0, 2 ** 64, 30_000, dtype=np.uint64)
    # keys exactly at / next to every range boundary ceil(r * 2^64 / G)
    for r in range(1, shards):
        b = -((-(r << 64)) // shards)
        pool[r * 3: r * 3 + 3] = [b - 1, b, min(b + 1, 2 ** 64 - 1)]
    keys = pool[rng.integers(0, len(pool), 90_001)]
    me = MultiEngine([0] * shards)
    cuts = [len(keys) * i // shards for i in range(shards + 1)]
    parts = [dev64(keys[cuts[i]:cuts[i + 1]]) for i in range(shards)]
    reps, objects = me.group(parts, cuts[:-1])
    orep, oobj = oracle.group_canonical(keys)
    assert objects == oobj
    got = np.concatenate([r.cpu().numpy() for r in reps])
    assert (got == orep.astype(np.int64)).all()
    me.close()


def test_multi_device_hash_group_host(eng, oracle):
    from spacedrive_amd.multi import MultiEngine
    rng = np.random.default_rng(30)
    n = 3001
    content = rng.integers(0, 256, (n, SAMPLED_CONTENT_LEN), dtype=np.uint8)
    sizes = rng.integers(MINIMUM_FILE_SIZE + 1, 2 ** 40, n, dtype=np.uint64)
    dup = rng.integers(0, n, 700)
    src = rng.integers(0, n, 700)
    content[dup] = content[src]
    sizes[dup] = sizes[src]
    want = oracle.fast_cas_keys_strided(content.reshape(-1), SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN, sizes, 8)
    orep, oobj = oracle.group_canonical(want)
    me = MultiEngine([0, 0, 0])
    keys, rep, objects = me.hash_group_sampled_host(content.reshape(-1), sizes)
    assert (keys == want).all()
    assert objects == oobj and (rep == orep.astype(np.uint64)).all()
    me.close()


@pytest.mark.gpu
def test_packed_layout_alignment_invariance(path_eng, oracle):
    """synth_small packs whole-file contents at 128-B lines (K2's line pair = one cache
    line); the same files at 16-B packed offsets (the ABI's minimum,
    written by sd_cas_synth_small_content_dev) give identical cas keys, equal to the
    oracle's, and so do the K1L shapes below the latency threshold."""
    eng = path_eng
    n = 20_000
    sz = torch.empty(n, dtype=torch.int64, device="cuda")
    ln = torch.empty(n, dtype=torch.int32, device="cuda")
    of = torch.empty(n, dtype=torch.int64, device="cuda")
    nb = eng.synth_small(91, 0, n, sz, ln, of, None)
    arena = torch.empty(nb + 64, dtype=torch.uint8, device="cuda")
    eng.synth_small(91, 0, n, sz, ln, of, arena)
    assert bool((of % 128 == 0).all())
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.hash_packed(arena, of, ln, sz, keys)
    lens = ln.cpu().numpy().astype(np.uint32)
    want = oracle.fast_cas_keys(arena.cpu().numpy(), of.cpu().numpy().astype(np.uint64), lens,
                                host64(sz), 8)
    assert (host64(keys) == want).all()
    al = (ln.to(torch.int64) + 15) // 16 * 16
    of16 = torch.cumsum(al, 0) - al
    arena16 = torch.empty(int(al.sum().item()) + 64, dtype=torch.uint8, device="cuda")
    eng.synth_small_content(91, 0, n, of16, ln, arena16)
    keys16 = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.hash_packed(arena16, of16, ln, sz, keys16)
    assert (host64(keys16) == want).all()
    for m in (100, 5_000):  # K1L one wave per file / four files per wave
        k = torch.empty(m, dtype=torch.int64, device="cuda")
        eng.hash_packed(arena16, of16[:m].contiguous(), ln[:m].contiguous(), sz[:m].contiguous(), k)
        assert (host64(k) == want[:m]).all()
