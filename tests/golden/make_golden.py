"""Generates tests/golden/golden.json — the committed golden vectors for the cas path.

Run:  python tests/golden/make_golden.py      (CPU only; uses the oracle, not the product)

Provenance of each section (see DESIGN.md "Parity"):
  * "derive_key_kat"   — copied from the reference's own test: DERIVE_B3_EXPECTED,
    crates/crypto/src/keys/hashing.rs:210-213 (test :323-328), material = KEY (0x23 x 32,
    :132-136) || SALT (0xFF x 16, :138-141), context :121.  Externally pinned.
  * "blake3_public"    — BLAKE3("") / BLAKE3("abc"), public values quoted in SURVEY.md §8c.
    Externally pinned.
  * "blake3_lengths"   — BLAKE3 of the i % 251 byte pattern at lengths straddling chunk and
    tree boundaries, produced by the C oracle and REQUIRED to agree with its recursive and
    level-wise formulations and with the independent pure-Python restatement.
  * "cas"              — cas_ids of synthetic files (content = splitmix64 stream keyed by
    (seed, file), shared with the device generator), sizes per SURVEY.md §8c, including the
    100 KiB threshold (cas.rs:27, inclusive) and a > 4 GiB file (virtual image: only the
    bytes at the cas.rs:35-58 offsets are generated).  Cross-checked C vs Python oracle.
  * "grouping"         — hand-built duplicate layouts with canonical reps and the literal
    replay of identifier_job_step (mod.rs:98-350) in 100-row chunks.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.pyoracle import (  # noqa: E402
    MINIMUM_FILE_SIZE,
    Oracle,
    np_file_key,
    np_mix64,
    py_blake3,
    py_cas_id,
    py_derive_key,
    py_sample_plan,
)

_G = np.uint64(0x9E3779B97F4A7C15)


def virtual_file_bytes(seed: int, file: int, off: int, length: int) -> bytes:
    """Bytes [off, off+length) of the synthetic file image (same stream as np_content)."""
    w0, w1 = off // 8, (off + length + 7) // 8
    key = np_file_key(seed, file)
    with np.errstate(over="ignore"):
        w = np_mix64(key + (np.arange(w0 + 1, w1 + 1, dtype=np.uint64) * _G))
    b = w.astype("<u8").tobytes()
    return b[off - 8 * w0: off - 8 * w0 + length]


def gather_virtual(seed: int, file: int, size: int) -> bytes:
    if size <= MINIMUM_FILE_SIZE:
        return virtual_file_bytes(seed, file, 0, size)
    return b"".join(virtual_file_bytes(seed, file, o, ln) for o, ln in py_sample_plan(size))


def replay_identifier(keys: list[int], chunk: int = 100):
    """Literal replay of identifier_job_step over a fresh library (mod.rs:98-350):
    Objects table in creation order; HashMap iteration := ascending idx."""
    objects = []          # list of (object_id, set of cas)
    cas_to_objs = {}      # cas -> [object ids] in creation order
    obj_of = {}
    created_total = linked_total = 0
    for c0 in range(0, len(keys), chunk):
        rows = list(range(c0, min(len(keys), c0 + chunk)))
        # :181-198 existing Objects whose file_paths carry any of this chunk's cas
        existing = {k: cas_to_objs[k] for k in {keys[i] for i in rows} if k in cas_to_objs}
        linked = []
        for i in rows:  # :202-238 link to the FIRST existing Object (lowest id)
            if keys[i] in existing:
                obj_of[i] = min(existing[keys[i]])
                linked.append(i)
        for i in rows:  # :246-311 one new Object per remaining file
            if keys[i] not in existing:
                oid = len(objects)
                objects.append(oid)
                obj_of[i] = oid
                cas_to_objs.setdefault(keys[i], []).append(oid)
                created_total += 1
        linked_total += len(linked)
    owner = {}
    for i in sorted(obj_of):
        owner.setdefault(obj_of[i], i)
    rep_chunked = [owner[obj_of[i]] for i in range(len(keys))]
    return rep_chunked, created_total, linked_total


ROW_HASHED, ROW_NO_CAS, ROW_ERROR = 0, 1, 2
LINK_CREATED, LINK_LINKED, LINK_DROPPED, LINK_NOT_REACHED, LINK_EXISTING = 0, 1, 2, 3, 4
NO_STEP = NO_OBJECT = 0xFFFFFFFF


def replay_identifier_job(keys, states, chunk: int = 100, with_creates: bool = False,
                          existing=None, pre_objects=None):
    """Literal replay of one file-identifier job, DB state included:
    file_identifier_job.rs:86-178 (init: orphan count, ceil(n/chunk) steps, cursor = first
    orphan id), :180-236 (execute_step: get_orphan_file_paths = orphan rows — object_id NULL
    OR cas_id NULL, :258-261 — with id >= cursor, ascending, LIMIT chunk (:251-319); an empty
    query ends the job), mod.rs:98-350 (identifier_job_step: FileMetadata per row, errors
    dropped; cas_id written; find_many = every Object connected to a file_path whose cas_id
    is one of the step's, in id order; each row links to the first that carries its cas_id;
    one new Object per remaining row, HashMap order := ascending row) and mod.rs:401-405 (the
    next cursor = the chunk's last row).
    Rows: file_path ids 0..n-1 with cas_id NULL at init; object_id NULL unless pre_objects.
    existing: None (a fresh library) or (cas key, Object id) pairs — Objects the library
    holds before the job, each connected to a file_path (outside the job's rows) with that
    cas.  pre_objects: None or per row the Object its file_path already holds (None / -1 /
    NO_OBJECT: none) — the watcher's "created empty, then written" rows
    (watcher/utils.rs:236-293, 473-490).  Pre-job Objects take the Object table's first rows
    in id order, so find_many returns them ahead of the job's own Objects (:181-188; the
    query has no location filter).  Which Objects a cas_id finds is recomputed from the
    file_path table at every step (a row re-linked away from its Object disconnects it).
    Returns (step[], object[], action[], [(created, linked)] per step) where object[i] is
    the row that created the Object row i is connected to, or (LINK_EXISTING) the id of the
    pre-job Object; with_creates: also the rows that created an Object in each step (a
    re-queried empty row appears in every step it was processed in)."""
    n = len(keys)
    none = (None, -1, NO_OBJECT)
    pre = [None if p in none else int(p) for p in pre_objects] if pre_objects is not None else [None] * n
    assert len(pre) == n
    pre_id = sorted({int(o) for _, o in existing or ()} | {p for p in pre if p is not None})
    pos = {oid: t for t, oid in enumerate(pre_id)}   # Object-table row of a pre-job Object
    creator = [None] * len(pre_id)  # Object table: position -> creating row (None: pre-job)
    cas_col = [None] * n            # file_path.cas_id
    obj_col = [None if p is None else pos[p] for p in pre]  # file_path.object_id (table row)
    conn = {}                       # cas -> {Object position: file_paths connecting them}

    def connect(cas, o, d):
        if cas is None or o is None:
            return
        m = conn.setdefault(cas, {})
        m[o] = m.get(o, 0) + d
        if m[o] == 0:
            del m[o]

    def update(r, cas=..., obj=...):  # one file_path UPDATE: keeps `conn` in step with the table
        connect(cas_col[r], obj_col[r], -1)
        if cas is not ...:
            cas_col[r] = cas
        if obj is not ...:
            obj_col[r] = obj
        connect(cas_col[r], obj_col[r], +1)

    for c, o in existing or ():     # the seeds' own file_paths (never job rows)
        connect(int(c), pos[int(o)], +1)
    step = [NO_STEP] * n
    processed_ok = [False] * n   # last processing of the row succeeded
    processed = [False] * n
    counts = []
    step_creates = []
    cursor = 0
    for k in range(-(-n // chunk) if chunk else 0):
        rows = []
        r = cursor
        while r < n and len(rows) < chunk:          # orphan: object_id NULL or cas_id NULL
            if obj_col[r] is None or cas_col[r] is None:
                rows.append(r)
            r += 1
        if not rows:
            break                                    # JobError::EarlyFinish
        meta = {}
        for r in rows:                               # FileMetadata::new (mod.rs:105-147)
            step[r] = k
            processed[r] = True
            processed_ok[r] = states[r] != ROW_ERROR
            if states[r] == ROW_ERROR:
                continue
            meta[r] = None if states[r] == ROW_NO_CAS else keys[r]
        for r, c in meta.items():                    # cas_id write (mod.rs:157-178)
            update(r, cas=c)
        unique = {c for c in meta.values() if c is not None}
        found = {c: sorted(conn[c]) for c in unique if conn.get(c)}  # :181-198, id order
        linked = 0
        for r in sorted(meta):                       # :202-238 link to the FIRST Object
            c = meta[r]
            if c is not None and c in found:
                update(r, obj=found[c][0])
                linked += 1
        created = 0
        step_creates.append([])
        for r in sorted(meta):                       # :246-347 one new Object per remaining row
            c = meta[r]
            if c is None or c not in found:
                creator.append(r)
                update(r, obj=len(creator) - 1)
                created += 1
                step_creates[-1].append(r)
        counts.append((created, linked))
        cursor = rows[-1]                            # mod.rs:401-405
    obj = [NO_OBJECT] * n
    act = [LINK_NOT_REACHED] * n
    for r in range(n):
        if not processed[r]:
            continue
        if not processed_ok[r]:
            act[r] = LINK_DROPPED
            continue
        if creator[obj_col[r]] is None:
            obj[r] = pre_id[obj_col[r]]
            act[r] = LINK_EXISTING
            continue
        obj[r] = creator[obj_col[r]]
        act[r] = LINK_CREATED if obj[r] == r else LINK_LINKED
    if with_creates:
        return step, obj, act, counts, step_creates
    return step, obj, act, counts


# ---- the link emission's closed form, vectorised (large jobs; sd_cas_identifier_links_ex):
# a hashed row's Object = min(seeds of its key, Objects of its key's rows in steps <= its own);
# else CREATED in its key's first step, LINKED to that first row after.  Equal to the literal
# replay above (tests/test_oracle.py::test_pre_object_closed_form_vs_replay pins the scalar
# form; tools/stress_links.py checks this one against the replay on small jobs).
_NONE = 0xFFFFFFFF


def cursor_walk(states, n, chunk):
    """Per-row final step (_NONE if unreached) and the job's step starts (the reference's
    `id >= cursor` query; a chunk's last row that stays orphan is queried again)."""
    steps_total = -(-n // chunk)
    starts = []
    start, reached = 0, 0
    for _ in range(steps_total):
        if start >= n:
            break
        starts.append(start)
        end = min(start + chunk, n)
        reached = end
        start = end - 1 if states[end - 1] != 0 else end
    step = np.full(n, _NONE, np.int64)
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else reached
        step[s:e] = k
    return step, starts, reached


def closed_form(keys, states, pre, seeds, step, starts=None):
    """Vectorised: per hashed row, min(seeds of its key, the Objects of its key's rows in
    steps <= its step); else CREATED in its key's first step, LINKED to the first row after."""
    n = len(keys)
    obj = np.full(n, _NONE, np.int64)
    act = np.full(n, 3, np.int64)
    act[(step != _NONE) & (states == 2)] = 2
    nc = (step != _NONE) & (states == 1)
    act[nc] = 0
    obj[nc] = np.flatnonzero(nc)
    rows = np.flatnonzero((states == 0) & (step != _NONE))
    if len(rows) == 0:
        return obj, act
    rows = rows[np.lexsort((rows, keys[rows]))]          # (key, row) order
    k = keys[rows]
    st = step[rows]
    m = len(rows)
    head = np.r_[True, k[1:] != k[:-1]]
    seg = np.cumsum(head) - 1
    first = rows[np.flatnonzero(head)][seg]
    # segmented running minimum of the rows' Objects (max-accumulate of seg * 2^33 + ~v)
    BIG = np.int64(1) << 33
    v = pre[rows].astype(np.int64)
    w = np.maximum.accumulate(seg.astype(np.int64) * BIG + (BIG - 1 - v))
    pm = BIG - 1 - (w - seg.astype(np.int64) * BIG)
    # value at the end of each (key, step) run
    end = np.flatnonzero(np.r_[(k[1:] != k[:-1]) | (st[1:] != st[:-1]), True])
    target = pm[end[np.searchsorted(end, np.arange(m))]]
    if seeds:
        sk = np.array([x for x, _ in seeds], np.uint64)
        so = np.array([o for _, o in seeds], np.int64)
        o2 = np.lexsort((so, sk))
        sk, so = sk[o2], so[o2]
        sh = np.r_[True, sk[1:] != sk[:-1]]
        uk, umin = sk[sh], so[sh]
        pos = np.searchsorted(uk, k)
        hit = (pos < len(uk)) & (uk[np.minimum(pos, len(uk) - 1)] == k)
        target = np.where(hit, np.minimum(target, umin[np.minimum(pos, len(uk) - 1)]), target)
    ex = target != _NONE
    obj[rows[ex]] = target[ex]
    act[rows[ex]] = 4
    cr = ~ex & (st == step[first])
    obj[rows[cr]] = rows[cr]
    act[rows[cr]] = 0
    ln = ~ex & ~cr
    obj[rows[ln]] = first[ln]
    act[rows[ln]] = 1
    return obj, act


def canonical(keys: list[int]):
    first = {}
    rep = []
    for i, k in enumerate(keys):
        first.setdefault(k, i)
        rep.append(first[k])
    return rep, len(first)


def main() -> None:
    o = Oracle()
    out: dict = {"generator": "tests/golden/make_golden.py"}
    material = bytes([0x23] * 32 + [0xFF] * 16)
    ctx = "spacedrive 2023-02-09 17:44:14 test key derivation"
    expected = bytes([27, 34, 251, 101, 201, 89, 78, 90, 20, 175, 62, 206, 200, 153, 166, 103,
                      118, 179, 194, 44, 216, 26, 48, 120, 137, 157, 60, 234, 234, 53, 46, 60])
    assert o.derive_key(ctx, material) == expected == py_derive_key(ctx, material)
    out["derive_key_kat"] = {"context": ctx, "material_hex": material.hex(), "expected_hex": expected.hex(),
                             "source": "crates/crypto/src/keys/hashing.rs:210-213,323-328"}
    # the reference's Balloon-BLAKE3 password-hash KATs (hashing.rs:58-65 params, :130
    # password, :138-141 salt, :143-146 secret, :180-208 expected; tests :269-321): reproduced
    # by oracle/balloon_ref.c, they pin BLAKE3 on streamed multi-block inputs
    balloon = {"password_hex": b"password".hex(), "salt_hex": "ff" * 16, "secret_hex": "55" * 18,
               "t_cost": 2, "p_cost": 1, "source": "crates/crypto/src/keys/hashing.rs:58-65,130-146,180-208",
               "vectors": []}
    b3b = [bytes([105, 36, 165, 219, 22, 136, 156, 19, 32, 143, 237, 150, 236, 194, 70, 113, 73, 137,
                  243, 106, 80, 31, 43, 73, 207, 210, 29, 251, 88, 6, 132, 77]),
           bytes([179, 71, 60, 122, 54, 72, 132, 209, 146, 96, 15, 115, 41, 95, 5, 75, 214, 135, 6, 122,
                  82, 42, 158, 9, 117, 19, 19, 40, 48, 233, 207, 237]),
           bytes([233, 60, 62, 184, 29, 152, 111, 46, 239, 126, 98, 90, 211, 255, 151, 0, 10, 189, 61,
                  84, 229, 11, 245, 228, 47, 114, 87, 74, 227, 67, 24, 141])]
    b3bs = [bytes([188, 0, 43, 39, 137, 199, 91, 142, 97, 31, 98, 6, 130, 75, 251, 71, 150, 109, 29, 62,
                   237, 171, 210, 22, 139, 108, 94, 190, 91, 74, 134, 47]),
            bytes([19, 247, 102, 192, 129, 184, 29, 147, 68, 215, 234, 146, 153, 221, 65, 134, 68, 120,
                   207, 209, 184, 246, 127, 131, 9, 245, 91, 250, 220, 61, 76, 248]),
            bytes([165, 240, 162, 25, 172, 3, 232, 2, 43, 230, 226, 128, 174, 28, 211, 61, 139, 136, 221,
                   197, 16, 83, 221, 18, 212, 190, 138, 79, 239, 148, 89, 215])]
    for k, s_cost in enumerate((131_072, 262_144, 524_288)):
        for sec, want in ((None, b3b[k]), (b"\x55" * 18, b3bs[k])):
            assert o.balloon_blake3(b"password", b"\xff" * 16, sec, s_cost, 2) == want, (s_cost, sec)
            balloon["vectors"].append({"s_cost": s_cost, "secret": sec is not None, "expected_hex": want.hex()})
    out["balloon_b3_kat"] = balloon
    pub = {"": "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
           "abc": "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85"}
    for s, h in pub.items():
        assert o.blake3(s.encode()).hex() == h == py_blake3(s.encode()).hex()
    out["blake3_public"] = pub

    lens = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 2049, 3072, 3073, 4096, 4097, 5120, 5121,
            6144, 6145, 7168, 7169, 8192, 8193, 16384, 31744, 57352, 65536, 102400, 102408, 140000]
    rows = []
    for n in lens:
        d = bytes(i % 251 for i in range(n))
        h = o.blake3(d)
        assert h == o.blake3_recursive(d) == o.blake3_levelwise(d), n
        if n <= 20000:
            assert h == py_blake3(d), n
        rows.append({"len": n, "hex": h.hex()})
    out["blake3_lengths"] = {"pattern": "byte i = i % 251", "vectors": rows}

    seed = 0x5DCA50001
    sizes = [1, 63, 64, 65, 1015, 1016, 1017, 1024, 2040, 102399, 102400, 102401, 102402,
             10 ** 6, (1 << 32) + 7]
    cas = []
    for f, s in enumerate(sizes):
        content = gather_virtual(seed, f, s)
        cid = o.cas_id(content, s)
        assert cid == py_cas_id(content, s), s
        cas.append({"file": f, "size": s, "content_len": len(content), "cas_id": cid,
                    "plan": py_sample_plan(s) if s > MINIMUM_FILE_SIZE else None})
    out["cas"] = {"seed": seed, "content": "splitmix64 words mix64(file_key(seed,file)+(w+1)*GAMMA), LE",
                  "files": cas}

    layouts = {}
    rng = np.random.default_rng(7)
    # (a) all distinct; (b) all identical; (c) pairs across a chunk edge; (d) dups inside
    # the first chunk + later links; (e) random 30 % duplicates over 350 files
    a = [int(x) for x in rng.integers(0, 2 ** 63, 250)]
    b = [0xDEADBEEF] * 230
    c = [int(x) for x in rng.integers(0, 2 ** 63, 220)]
    c[150] = c[99]; c[100] = c[99]; c[201] = c[0]
    d = [int(x) for x in rng.integers(0, 2 ** 63, 300)]
    d[5] = d[3]; d[7] = d[3]; d[120] = d[3]; d[250] = d[5]; d[299] = d[98]
    e = []
    for i in range(350):
        e.append(e[int(rng.integers(0, i))] if i and rng.random() < 0.3 else int(rng.integers(0, 2 ** 64, dtype=np.uint64)))
    for name, keys in {"distinct": a, "identical": b, "chunk_edge": c, "first_chunk_dups": d,
                       "dup30": e}.items():
        rep, objs = canonical(keys)
        rc, created, linked = replay_identifier(keys)
        orep, oobjs = o.group_canonical(np.array(keys, dtype=np.uint64))
        assert list(orep) == rep and oobjs == objs, name
        crep, cc, cl = o.group_chunked(np.array(keys, dtype=np.uint64), 100)
        assert list(crep) == rc and cc == created and cl == linked, name
        layouts[name] = {"keys": [f"{k:016x}" for k in keys], "rep": rep, "objects": objs,
                         "rep_chunked": rc, "created": created, "linked": linked}
    out["grouping"] = {"chunk": 100, "layouts": layouts}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
