"""CPU tests: the oracle against the golden vectors and the reference's own KAT.

The oracle is a restatement of the reference path (oracle/oracle.h); before any GPU
parity claim rests on it, it is pinned here:
  * derive_key KAT from crates/crypto/src/keys/hashing.rs:210-213 (the reference's only
    in-repo BLAKE3 known answer),
  * public BLAKE3("") / BLAKE3("abc"),
  * multi-chunk trees (1-128 chunks, every chunk count) against an independent BLAKE3 in the
    image (hf_xet's Rust crate; tests/golden/make_xet_vectors.py),
  * every tree shape up to 1 GiB, the cas messages, keyed/derive_key modes and file_checksum
    against the BLAKE3 team's C implementation (1.8.2, exported by ROCm's libclang-cpp.so;
    tests/ext_blake3.py),
  * three independent tree formulations + a pure-Python restatement agreeing,
  * cas.rs:35-58 offsets simulated literally,
  * grouping against a literal replay of identifier_job_step (mod.rs:98-350).
"""
import os

import numpy as np
import pytest

from oracle.pyoracle import (
    MINIMUM_FILE_SIZE,
    SAMPLED_CONTENT_LEN,
    np_content,
    py_blake3,
    py_cas_id,
    py_derive_key,
    py_sample_plan,
)
from tests.golden.make_golden import canonical, gather_virtual, replay_identifier


def test_derive_key_kat_from_reference(oracle, golden):
    kat = golden["derive_key_kat"]
    mat = bytes.fromhex(kat["material_hex"])
    assert oracle.derive_key(kat["context"], mat).hex() == kat["expected_hex"]
    assert py_derive_key(kat["context"], mat).hex() == kat["expected_hex"]


def test_balloon_b3_kats_from_reference(oracle, golden):
    """The reference's other BLAKE3 known answers: Balloon::<blake3::Hasher> password hashes
    (crates/crypto/src/keys/hashing.rs:180-208, tests :269-321) — millions of streamed
    multi-piece BLAKE3 inputs of one and two 64-B blocks, so they pin the chunk-internal block
    chaining that the one-block derive_key vector does not.  The standard-params vectors run
    here (~1 s each); all six were reproduced by tests/golden/make_golden.py."""
    g = golden["balloon_b3_kat"]
    pwd, salt, sec = (bytes.fromhex(g[k]) for k in ("password_hex", "salt_hex", "secret_hex"))
    assert pwd == b"password" and salt == b"\xff" * 16 and sec == b"\x55" * 18
    assert len(g["vectors"]) == 6
    for v in g["vectors"]:
        if v["s_cost"] != 131_072:
            continue
        got = oracle.balloon_blake3(pwd, salt, sec if v["secret"] else None, v["s_cost"], g["t_cost"])
        assert got.hex() == v["expected_hex"], v


def _xet_vectors():
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "xet_blake3.json")) as f:
        return json.load(f)


def test_blake3_trees_pinned_by_independent_blake3(oracle):
    """Multi-chunk trees: every chunk count 1..128 with a ragged last chunk, plus the sampled
    cas message (57,352 B) and the largest whole-file one (102,408 B), each reproduced from
    digests hf_xet 1.5.2's Rust BLAKE3 computed on single-Xet-chunk files
    (tests/golden/make_xet_vectors.py has the relation).  The C oracle's keyed mode runs
    formulation 1's tree, the pure-Python restatement its own recursive tree."""
    import zlib

    from oracle.pyoracle import py_keyed_hash
    from tests.golden.make_xet_vectors import DATA_KEY, content, xet_display
    doc = _xet_vectors()
    assert doc["data_key"] == DATA_KEY.hex() and doc["unpinned"] == []
    lens = [v["len"] for v in doc["vectors"]]
    chunks = {-(-n // 1024) for n in lens}
    assert chunks == set(range(1, 129)) and {57_352, 102_408} <= set(lens)
    for i, v in enumerate(doc["vectors"]):
        d = content(v["len"], v["seed"])
        assert zlib.crc32(d) == v["crc32"], v
        inner = oracle.keyed_hash(DATA_KEY, d)
        assert xet_display(oracle.keyed_hash(bytes(32), inner)) == v["xet_hash"], v
        if i % 9 == 0:  # the pure-Python tree on a spread of lengths
            assert py_keyed_hash(DATA_KEY, d) == inner, v


def test_blake3_live_against_hf_xet(oracle, tmp_path):
    """Fresh draws (lengths 1..8 KiB, below Xet's minimum chunk, so always one Xet chunk)
    hashed live by hf_xet and by the oracle."""
    hf_xet = pytest.importorskip("hf_xet")
    from tests.golden.make_xet_vectors import DATA_KEY, xet_display
    rng = np.random.default_rng(2718)  # fixed: deterministic, still hashed live by hf_xet
    draws = []
    for i in range(24):
        d = rng.integers(0, 256, int(rng.integers(1, 8192)), dtype=np.uint8).tobytes()
        p = tmp_path / f"{i}.bin"
        p.write_bytes(d)
        draws.append((str(p), d))
    for (p, d), r in zip(draws, hf_xet.hash_files([p for p, _ in draws])):
        assert r.hash == xet_display(oracle.keyed_hash(bytes(32), oracle.keyed_hash(DATA_KEY, d))), len(d)


needs_ext = pytest.mark.skipif(not __import__("tests.ext_blake3").ext_blake3.available(),
                               reason="no libclang-cpp.so with the BLAKE3 C API in this image")


@needs_ext
def test_independent_c_blake3_binding(golden):
    """The binding itself: public vectors and the reference's derive_key KAT
    (crates/crypto/src/keys/hashing.rs:210-213) through the BLAKE3 team's C code."""
    from tests import ext_blake3 as ext
    assert ext.version().count(".") == 2
    for s_, h in golden["blake3_public"].items():
        assert ext.blake3(s_.encode()).hex() == h
    kat = golden["derive_key_kat"]
    assert ext.derive_key(kat["context"], bytes.fromhex(kat["material_hex"])).hex() == kat["expected_hex"]


@needs_ext
def test_oracle_trees_vs_independent_c_blake3(oracle, golden):
    """Every tree shape the product builds, oracle vs the BLAKE3 team's C implementation:
    the committed boundary lengths, every chunk count 1..300 with a ragged last chunk, 2^k
    chunks and one byte either side up to 64 MiB (all four formulations where they are
    fast), and a 1 GiB + 12,345-byte buffer through the threaded tree."""
    from tests import ext_blake3 as ext
    rng = np.random.default_rng(77)
    buf = rng.integers(0, 256, (1 << 26) + 2, dtype=np.uint8)
    lens = {r["len"] for r in golden["blake3_lengths"]["vectors"]}
    lens |= {(c - 1) * 1024 + int(rng.integers(1, 1025)) for c in range(1, 301)}
    for k in range(0, 17):
        lens |= {1024 * 2 ** k - 1, 1024 * 2 ** k, 1024 * 2 ** k + 1}
    for n in sorted(lens):
        d = buf[:n].tobytes()
        want = ext.blake3(d)
        assert oracle.blake3(d) == want, n
        if n <= 1 << 20:
            assert oracle.blake3_recursive(d) == want and oracle.blake3_levelwise(d) == want, n
        if n >= 1 << 22:
            assert oracle.blake3_mt(buf[:n], 8) == want, n
    big = rng.integers(0, 256, (1 << 30) + 12_345, dtype=np.uint8)
    assert oracle.blake3_mt(big, 8) == ext.blake3(big)


@needs_ext
def test_oracle_cas_keyed_and_checksum_vs_independent_c_blake3(oracle, tmp_path):
    """cas.rs's message (le64(size) || content) for both paths, the keyed mode the Xet
    vectors use, and file_checksum (hash.rs's 1 MiB read loop) against the C implementation."""
    from tests import ext_blake3 as ext
    rng = np.random.default_rng(78)
    for _ in range(200):
        size = int(rng.integers(1, 2 ** 40)) if rng.random() < 0.5 else int(rng.integers(1, 102_401))
        clen = SAMPLED_CONTENT_LEN if size > MINIMUM_FILE_SIZE else size
        c = rng.integers(0, 256, clen, dtype=np.uint8).tobytes()
        assert oracle.cas_key(c, size) == ext.cas_key(c, size), size
    for n in [1, 1024, 1025, 65_537, 131_072]:
        key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.keyed_hash(key, d) == ext.keyed_hash(key, d), n
    for n in [0, 1, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, 5 * (1 << 20) + 3]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        p = tmp_path / f"f{n}"
        p.write_bytes(d)
        assert oracle.file_checksum(str(p)) == ext.blake3(d).hex(), n


@needs_ext
def test_ext_b3_harness_matches_oracle(oracle):
    """bench.py's second CPU leg (oracle/ext_b3.c: the C implementation run through cas.rs's
    per-file sequence on pthreads) computes the same keys as the oracle's AVX-512 port."""
    from oracle.pyoracle import ExtBlake3
    ext = ExtBlake3()
    rng = np.random.default_rng(79)
    n = 300
    arena = rng.integers(0, 256, n * SAMPLED_CONTENT_LEN, dtype=np.uint8)
    sizes = rng.integers(MINIMUM_FILE_SIZE + 1, 2 ** 40, n, dtype=np.uint64)
    want = oracle.fast_cas_keys_strided(arena, SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN, sizes, 4)
    for threads in (1, 3, 8):
        got = ext.cas_keys_strided(arena, SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN, sizes, threads)
        assert (got == want).all(), threads
    assert ext.version().count(".") == 2


@needs_ext
def test_ext_b3_path_forms_match_oracle(oracle, tmp_path):
    """The paths legs of the CPU baselines (oracle/ext_b3.c): hash.rs's streamed loop and
    cas.rs's reads + the C library's hashing agree with the oracle file by file."""
    from oracle.pyoracle import ExtBlake3
    ext = ExtBlake3()
    rng = np.random.default_rng(80)
    paths, sizes = [], []
    for i, n in enumerate([0, 1, 1000, 102_400, 102_401, (1 << 20) - 1, 1 << 20, (1 << 20) + 1,
                           3 * (1 << 20) + 5]):
        p = tmp_path / f"f{i}"
        p.write_bytes(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        paths.append(str(p))
        sizes.append(n)
    paths.append(str(tmp_path / "missing"))
    sizes.append(5)
    for threads in (1, 4):
        hexes, errs = ext.file_checksums(paths, threads)
        for p, h, e in zip(paths, hexes, errs):
            if p.endswith("missing"):
                assert h is None and e == 2
            else:
                assert h == oracle.file_checksum(p) == ext.file_checksum(p), p
        keys, st = ext.cas_keys_paths(paths, sizes, threads)
        want, wst = oracle.generate_cas_keys_paths(paths, sizes, 2)
        assert (keys[:-1] == want[:-1]).all() and st[-1] == wst[-1] != 0


def test_public_vectors(oracle, golden):
    for s, h in golden["blake3_public"].items():
        assert oracle.blake3(s.encode()).hex() == h
        assert py_blake3(s.encode()).hex() == h


def test_length_vectors_three_formulations(oracle, golden):
    for row in golden["blake3_lengths"]["vectors"]:
        d = bytes(i % 251 for i in range(row["len"]))
        assert oracle.blake3(d).hex() == row["hex"]
        assert oracle.blake3_recursive(d).hex() == row["hex"]
        assert oracle.blake3_levelwise(d).hex() == row["hex"]


@pytest.mark.parametrize("n", [0, 1, 64, 1024, 1025, 3000, 8193])
def test_python_restatement_agrees(oracle, n):
    d = np_content(11, n, n)
    assert py_blake3(d) == oracle.blake3(d)


def test_formulations_random_lengths(oracle):
    rng = np.random.default_rng(3)
    for n in rng.integers(0, 300_000, 40):
        d = rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()
        a = oracle.blake3(d)
        assert a == oracle.blake3_recursive(d) == oracle.blake3_levelwise(d)


def test_sample_plan_matches_literal_loop(oracle):
    # cas.rs:35-58: header at 0, samples at 8192 + k*jump, footer at size - 8192
    for size in [102401, 102402, 123457, 10 ** 6, 2 ** 31 + 5, 2 ** 40 + 3]:
        plan = py_sample_plan(size)
        assert plan == oracle.sample_plan(size)
        jump = (size - 2 * 8192) // 4
        assert plan == [(0, 8192)] + [(8192 + k * jump, 10240) for k in range(4)] + [(size - 8192, 8192)]
        assert sum(ln for _, ln in plan) == SAMPLED_CONTENT_LEN


def test_golden_cas_ids(oracle, golden):
    g = golden["cas"]
    for f in g["files"]:
        content = gather_virtual(g["seed"], f["file"], f["size"])
        assert len(content) == f["content_len"]
        assert oracle.cas_id(content, f["size"]) == f["cas_id"]
        assert py_cas_id(content, f["size"]) == f["cas_id"]
        # inclusive 100 KiB threshold (cas.rs:27)
        assert (f["content_len"] == f["size"]) == (f["size"] <= MINIMUM_FILE_SIZE)


def test_gather_from_files_matches_image(oracle, tmp_path):
    rng = np.random.default_rng(5)
    for size in [0, 1, 100, 102400, 102401, 300_000, 1_000_003]:
        img = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        p = tmp_path / f"f{size}"
        p.write_bytes(img)
        got = oracle.gather_path(str(p), size)
        want = img if size <= MINIMUM_FILE_SIZE else b"".join(img[o:o + ln] for o, ln in py_sample_plan(size))
        assert got == want
        assert oracle.generate_cas_id(str(p), size) == oracle.cas_id(want, size)


def test_paths_baseline_matches_single_file(oracle, tmp_path):
    """The all-cores config-1 CPU baseline equals generate_cas_id file by file."""
    rng = np.random.default_rng(6)
    paths, sizes = [], []
    for i, size in enumerate([0, 7, 4096, 102400, 102401, 500_000] * 3 + [300_000] * 40):
        p = tmp_path / f"p{i}"
        p.write_bytes(rng.integers(0, 256, size, dtype=np.uint8).tobytes())
        paths.append(str(p)); sizes.append(size)
    paths.append(str(tmp_path / "missing")); sizes.append(10)
    for threads, simd in ((1, False), (4, False), (1, True), (3, True)):
        keys, status = oracle.generate_cas_keys_paths(paths, sizes, threads, simd)
        assert status[-1] == -2 and keys[-1] == 0
        assert [f"{k:016x}" for k in keys[:-1]] == [oracle.generate_cas_id(p, s)
                                                     for p, s in zip(paths[:-1], sizes[:-1])]


def test_gather_short_file_is_eof_error(oracle, tmp_path):
    p = tmp_path / "short"
    p.write_bytes(b"x" * 150_000)
    with pytest.raises(OSError):
        oracle.gather_path(str(p), 10 ** 7)  # size from stale metadata: read_exact -> EOF


STALE_SAMPLED = [  # (actual length on disk, fs::metadata size the caller passes)
    (300_000, 250_000),     # grew: samples from `size`, footer from the actual end
    (5_000_000, 200_000),   # grew a lot
    (240_000, 250_000),     # shrank, every sample still in bounds: a cas_id
    (230_000, 1_000_000),   # shrank below the 2nd sample: UnexpectedEof
    (60_000, 150_000),      # shrank below the last sample: UnexpectedEof
    (150_000, 150_000),     # unchanged
]


def stale_files(tmp_path):
    rng = np.random.default_rng(15)
    out = []
    for j, (actual, size) in enumerate(STALE_SAMPLED):
        p = tmp_path / f"stale_sampled{j}"
        p.write_bytes(rng.integers(0, 256, actual, dtype=np.uint8).tobytes())
        out.append((str(p), size))
    return out


def test_sampled_footer_follows_actual_end(oracle, tmp_path):
    """cas.rs:54-55 seeks SeekFrom::End(-8192): the footer of a file whose length changed
    since fs::metadata comes from its ACTUAL end.  The C oracle's pread gather must agree
    with a literal execution of the reference's read/seek sequence on the same files,
    including which stale files fail with UnexpectedEof (-EIO)."""
    from oracle.pyoracle import UnexpectedEof, py_generate_cas_id_file
    for path, size in stale_files(tmp_path):
        try:
            want = py_generate_cas_id_file(path, size)
        except UnexpectedEof:
            want = None
        if want is None:
            with pytest.raises(OSError) as ei:
                oracle.generate_cas_id(path, size)
            assert ei.value.errno == 5, (path, size)
        else:
            assert oracle.generate_cas_id(path, size) == want, (path, size)
    # the grown file's footer is NOT the one at size - 8192
    path, size = stale_files(tmp_path)[0]
    img = open(path, "rb").read()
    at_size = oracle.cas_id(b"".join(img[o:o + ln] for o, ln in py_sample_plan(size)), size)
    assert oracle.generate_cas_id(path, size) != at_size


def test_file_checksum(oracle, tmp_path):
    for n in [0, 1, 1024, 1025, 1 << 20, (1 << 20) + 17]:
        d = np_content(9, n, n)
        p = tmp_path / f"c{n}"
        p.write_bytes(d)
        assert oracle.file_checksum(str(p)) == oracle.blake3(d).hex()


def test_tree_parallel_modes_agree(oracle, tmp_path):
    """The multithreaded tree (16 MiB subtrees merged by pair-and-promote) equals the
    sequential hash at lengths around the subtree and chunk boundaries; the generated
    stream mode equals hashing the materialised stream; the file mode equals the literal
    file_checksum loop."""
    sub = 16 << 20
    for L in [0, 1, 1024, sub - 1, sub, sub + 1, sub + 1024, 2 * sub, 3 * sub + 777, 5 * sub - 1025]:
        d = oracle.fill_content_range(41, 2, 0, L)
        want = oracle.blake3(d.tobytes())
        assert oracle.blake3_mt(d, 4) == want, L
        assert oracle.stream_blake3_mt(41, 2, L, 3) == want, L
        if L in (sub + 1, 3 * sub + 777):
            p = tmp_path / "mt.bin"
            p.write_bytes(d.tobytes())
            assert oracle.file_checksum_mt(str(p), 4) == want.hex() == oracle.file_checksum(str(p))
    # the stream at an unaligned offset equals the slice of the materialised stream
    d = oracle.fill_content_range(41, 2, 0, 5000)
    assert (oracle.fill_content_range(41, 2, 13, 4000) == d[13:4013]).all()
    assert oracle.fill_content(41, 2, 5000) == d.tobytes()


def test_file_checksum_reads_to_eof_not_stat(oracle):
    """hash.rs:15-21 reads until the first short read, whatever fstat says: a procfs file
    with st_size 0 but content is hashed over its content."""
    p = "/proc/sys/kernel/ostype"
    if not os.path.exists(p) or os.stat(p).st_size != 0:
        pytest.skip("no procfs file with st_size 0")
    content = open(p, "rb").read()
    assert content and oracle.file_checksum(p) == oracle.blake3(content).hex()


def test_grouping_golden(oracle, golden):
    g = golden["grouping"]
    for name, lay in g["layouts"].items():
        keys = np.array([int(k, 16) for k in lay["keys"]], dtype=np.uint64)
        rep, objs = oracle.group_canonical(keys)
        assert list(rep) == lay["rep"] and objs == lay["objects"], name
        rc, c, ln = oracle.group_chunked(keys, g["chunk"])
        assert list(rc) == lay["rep_chunked"] and (c, ln) == (lay["created"], lay["linked"]), name


def test_grouping_random_vs_replay(oracle):
    rng = np.random.default_rng(11)
    for trial in range(20):
        n = int(rng.integers(1, 700))
        pool = rng.integers(0, 2 ** 64, max(1, n // int(rng.integers(1, 6))), dtype=np.uint64)
        keys = pool[rng.integers(0, len(pool), n)]
        rep, objs = canonical([int(k) for k in keys])
        orep, oobjs = oracle.group_canonical(keys)
        assert list(orep) == rep and oobjs == objs
        rc, c, ln = replay_identifier([int(k) for k in keys], 100)
        crep, cc, cl = oracle.group_chunked(keys, 100)
        assert list(crep) == rc and (cc, cl) == (c, ln)


def test_job_replay_cursor_semantics():
    """The literal job replay (DB state + cursor): with every row hashed it equals the
    chunk replay; a row that stays orphan at a chunk's end (error / empty file) is queried
    again by the next step (mod.rs:401-405 + `id >= cursor`, file_identifier_job.rs:268),
    shifting every later chunk by one, and the job still runs only ceil(n/chunk) steps."""
    from tests.golden.make_golden import replay_identifier_job
    rng = np.random.default_rng(12)
    keys = [int(k) for k in rng.integers(0, 2 ** 63, 350)]
    keys[150] = keys[20]
    keys[260] = keys[120]
    step, obj, act, counts = replay_identifier_job(keys, [0] * 350, 100)
    rc, created, linked = replay_identifier(keys, 100)
    assert obj == rc and tuple(map(sum, zip(*counts))) == (created, linked)
    assert step == [i // 100 for i in range(350)]
    # row 99 errors: step 1 re-queries it and covers rows 99..198; row 198 is empty: step 2
    # re-queries it (a second new Object), rows 198..297; step 3 covers 298..349 only
    states = [0] * 300
    states[99], states[198] = 2, 1
    step, obj, act, counts = replay_identifier_job(keys[:300], states, 100)
    assert step[99] == 1 and act[99] == 2 and obj[99] == 0xFFFFFFFF
    assert step[198] == 2 and act[198] == 0 and obj[198] == 198
    assert step[199] == 2 and step[297] == 2 and len(counts) == 3
    assert step[298] == 0xFFFFFFFF and act[298] == act[299] == 3  # past the 3 steps: not reached
    assert counts[0] == (99, 0) and counts[1][0] + counts[1][1] == 99
    assert counts[2][0] + counts[2][1] == 100 + 0  # 198 again (new Object) + 199..297


def test_job_replay_existing_objects():
    """The replay on a library that already holds Objects (mod.rs:180-253): a row whose cas
    an older Object carries links to the lowest such Object id in every step and never
    creates; keys without one keep the fresh-library behaviour (no intra-step dedup, later
    steps link to the first creator)."""
    from tests.golden.make_golden import LINK_EXISTING, replay_identifier_job
    A, B, C, D = 0xA0, 0xB0, 0xC0, 0xD0
    keys = [A, C, B, C, A, D, A, C, B, D]
    states = [0, 0, 0, 0, 1, 0, 0, 0, 2, 0]
    existing = [(A, 7), (B, 12), (A, 3), (A, 9)]
    step, obj, act, counts = replay_identifier_job(keys, states, 4, existing=existing)
    assert step == [0, 0, 0, 0, 1, 1, 1, 1, 2, 2]
    assert act[0] == act[6] == LINK_EXISTING and obj[0] == obj[6] == 3  # A -> id 3 (lowest)
    assert act[2] == LINK_EXISTING and obj[2] == 12                     # B -> 12
    assert act[1] == act[3] == 0 and obj[3] == 3                        # C twice in step 0: two Objects
    assert act[7] == 1 and obj[7] == 1                                  # later C: the first one
    assert act[4] == 0 and obj[4] == 4                                  # no cas_id: own Object
    assert act[5] == 0 and act[9] == 1 and obj[9] == 5 and act[8] == 2  # D fresh; B errors
    assert counts == [(2, 2), (2, 2), (0, 1)]
    # unseeded: the same rows as a fresh library
    _, obj0, act0, _ = replay_identifier_job(keys, states, 4)
    assert act0[0] == 0 and obj0[6] == 0 and act0[2] == 0


def test_job_replay_rows_owning_objects():
    """Rows that already own an Object (object_id set, cas_id NULL — orphan by
    file_identifier_job.rs:258-261; the watcher's "created empty, then written" file,
    watcher/utils.rs:236-293,473-490): the step writes the row's cas_id before find_many
    (mod.rs:157-198), so the row's Object joins its key's Objects in that step; every row of
    the step with the key links to the smallest such id and the key never creates there; a
    pre-job Object takes over a key an earlier step created an Object for; a NO_CAS row with
    an Object still creates, an ERROR row keeps it (dropped)."""
    from tests.golden.make_golden import LINK_DROPPED, LINK_EXISTING, replay_identifier_job
    A, B, C, D, E = 0xA0, 0xB0, 0xC0, 0xD0, 0xE0
    keys = [A, B, A, C, A, B, D, A, C, A, E, B, A, 0, 0, A]
    states = [0] * 12 + [0, 1, 2, 0]
    pre = [None, None, None, 50, None, 20, None, None, None, 10, None, None, 60, 70, 80, None]
    step, obj, act, counts = replay_identifier_job(keys, states, 4, pre_objects=pre)
    assert step == [k // 4 for k in range(16)]
    assert act[:3] == [0, 0, 0] and (act[3], obj[3]) == (LINK_EXISTING, 50)  # C: its own Object
    assert (act[4], obj[4]) == (1, 0) and (act[7], obj[7]) == (1, 0)          # A: row 0's
    assert (act[5], obj[5]) == (LINK_EXISTING, 20)  # B: 20 is older than row 1's Object
    assert (act[8], obj[8]) == (LINK_EXISTING, 50)
    assert (act[9], obj[9]) == (LINK_EXISTING, 10)  # A taken over by the pre-job Object 10
    assert (act[11], obj[11]) == (LINK_EXISTING, 20) and act[10] == 0
    assert (act[12], obj[12]) == (LINK_EXISTING, 10)  # its own 60 loses to 10
    assert (act[13], obj[13]) == (0, 13) and act[14] == LINK_DROPPED
    assert (act[15], obj[15]) == (LINK_EXISTING, 10)
    assert counts == [(3, 1), (1, 3), (1, 3), (1, 2)]
    # without the pre-existing Objects: the fresh-library answer
    _, obj0, act0, _ = replay_identifier_job(keys, states, 4)
    assert act0[3] == 0 and (act0[9], obj0[9]) == (1, 0)


def closed_form_links(keys, states, step, chunk, existing=(), pre=None):
    """The per-row formula the GPU emission evaluates (links.hip), from the rows' steps:
    a hashed row's Object is the smallest pre-job Object carrying its key that the step
    sees — seeds, or pre-existing Objects of rows with the key in this or an earlier step —
    else the Object created for the key's first row (CREATED in that row's step)."""
    n = len(keys)
    NONE = 0xFFFFFFFF
    seedmin, first, ev = {}, {}, {}
    for c, o in existing:
        seedmin[c] = min(seedmin.get(c, NONE), o)
    for i in range(n):
        if step[i] != NONE and states[i] == 0:
            first.setdefault(keys[i], i)
            if pre is not None and pre[i] is not None:
                ev.setdefault(keys[i], []).append((step[i], pre[i]))
    obj, act = [NONE] * n, [3] * n
    for i in range(n):
        if step[i] == NONE:
            continue
        if states[i] == 2:
            act[i] = 2
        elif states[i] == 1:
            act[i], obj[i] = 0, i
        else:
            k = keys[i]
            v = min([seedmin.get(k, NONE)] + [p for s, p in ev.get(k, ()) if s <= step[i]])
            if v != NONE:
                act[i], obj[i] = 4, v
            elif step[first[k]] == step[i]:
                act[i], obj[i] = 0, i
            else:
                act[i], obj[i] = 1, first[k]
    return obj, act


def test_vectorised_closed_form_vs_replay():
    """The vectorised closed form the large GPU link tests check against
    (tests/golden/make_golden.py::closed_form, cursor_walk) equals the literal replay on 150
    random jobs: chunk 1..19, NO_CAS / ERROR rows, rows owning Objects, seeds."""
    from tests.golden.make_golden import closed_form, cursor_walk, replay_identifier_job
    rng = np.random.default_rng(33)
    for it in range(150):
        n = int(rng.integers(1, 300))
        chunk = int(rng.integers(1, 20))
        keys = rng.integers(1, max(2, n // 3), n).astype(np.uint64)
        states = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.9, 0.05, 0.05])
        pre = np.full(n, 0xFFFFFFFF, np.uint32)
        m = rng.random(n) < 0.2
        pre[m] = rng.permutation(10 * n + 40)[:int(m.sum())]
        uk = np.unique(keys)
        seeds = [(int(k), int(10 * n + 100 + j)) for j, k in enumerate(uk[rng.random(len(uk)) < 0.2])]
        step, starts, _ = cursor_walk(states, n, chunk)
        o, a = closed_form(keys, states, pre, seeds, step, starts)
        ws, wo, wa, _ = replay_identifier_job([int(k) for k in keys], [int(x) for x in states], chunk,
                                              existing=seeds,
                                              pre_objects=[None if x == 0xFFFFFFFF else int(x) for x in pre])
        assert (np.array(ws) == step).all() and (np.array(wo) == o).all() and (np.array(wa) == a).all(), it


@pytest.mark.parametrize("chunk", [100, 7, 3, 1])
def test_pre_object_closed_form_vs_replay(chunk):
    """The closed form behind sd_cas_identifier_links_ex (per-key prefix minimum over steps)
    equals the literal DB replay: random keys with repeats inside and across chunks, ~10 %
    of rows owning an Object (ids interleaved with the seeds'), seeds, NO_CAS / ERROR rows
    at chunk ends (the cursor re-queries them)."""
    from tests.golden.make_golden import replay_identifier_job
    rng = np.random.default_rng(400 + chunk)
    for trial in range(4):
        n = 700 if chunk > 2 else 300
        pool = [int(x) for x in rng.integers(1, 2 ** 63, max(4, n // (3 + trial)))]
        keys = [pool[int(j)] for j in rng.integers(0, len(pool), n)]
        states = [int(s) for s in rng.choice([0, 1, 2], n, p=[0.88, 0.06, 0.06])]
        if chunk == 1:  # a row that stays orphan is re-queried until the step budget ends
            states = [0] * (n - 3) + [1, 0, 2]
        ids = rng.permutation(4 * n)
        pre = [int(ids[i]) if rng.random() < 0.1 else None for i in range(n)]
        existing = [(pool[int(j)], int(ids[2 * n + t])) for t, j in
                    enumerate(rng.integers(0, len(pool), len(pool) // 4 * (trial % 2)))]
        step, obj, act, _ = replay_identifier_job(keys, states, chunk, existing=existing,
                                                  pre_objects=pre)
        cobj, cact = closed_form_links(keys, states, step, chunk, existing, pre)
        assert cact == act and cobj == obj, (chunk, trial)
        assert 4 in act


def test_simd_baseline_matches_scalar(oracle):
    rng = np.random.default_rng(2)
    n = 48
    arena = rng.integers(0, 256, n * SAMPLED_CONTENT_LEN, dtype=np.uint8)
    sizes = rng.integers(102401, 2 ** 32, n, dtype=np.uint64)
    a = oracle.cas_keys_strided(arena, SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN, sizes)
    b = oracle.fast_cas_keys_strided(arena, SAMPLED_CONTENT_LEN, SAMPLED_CONTENT_LEN, sizes, threads=2)
    assert (a == b).all()
    for L in [0, 55, 56, 57, 1016, 1017, 4000, 102400]:
        ar = rng.integers(0, 256, 16 * max(L, 1) + 64, dtype=np.uint8)
        offs = np.arange(16, dtype=np.uint64) * L
        ln = np.full(16, L, dtype=np.uint64)
        assert (oracle.cas_keys(ar, offs, ln, ln) == oracle.fast_cas_keys(ar, offs, ln, ln)).all()
    # unequal lengths in a group: chunk-parallel path (16 chunks of one file per lane
    # group, the tail chunk a masked lane, SIMD parent levels) — lengths straddle the
    # chunk, 16-chunk-group and 128-chunk (scalar) boundaries
    lens = np.array([1016, 1017, 2040, 2041, 16376, 16377, 17400, 32773, 102399, 102400,
                     63, 5000, 131064, 131065, 50000, 16 * 1024 * 3 - 8], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]]).astype(np.uint64)
    ar = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    sz = lens + rng.integers(0, 3, 16, dtype=np.uint64)  # size prefix need not equal the length
    assert (oracle.cas_keys(ar, offs, lens, sz) == oracle.fast_cas_keys(ar, offs, lens, sz, threads=2)).all()


def test_synth_generator_shared_definitions(oracle):
    # the device generator (spacedrive_amd/csrc/synth.hip) uses these exact definitions
    for f in [0, 1, 77, 10 ** 6]:
        assert oracle.fill_content(3, f, 1000) == np_content(3, f, 1000)
