#!/usr/bin/env python3
"""Generate tests/golden/xet_blake3.json: BLAKE3 tree vectors from an independent BLAKE3 in
this image (test infrastructure; run here, never on the GPU box).

The reference hashes with the external `blake3` 1.5.0 crate (Cargo.lock:1127-1139), which is
not vendored; the in-repo known answers pin one-chunk inputs only (derive_key KAT,
crates/crypto/src/keys/hashing.rs:210-213, and the Balloon KATs, hashing.rs:180-208).
The `hf_xet` wheel in this image (1.5.2, a Rust extension built on the `blake3` crate) exposes
`hash_files(paths)`, the Xet content hash of a file.  For a file that Xet's content-defined
chunker keeps as ONE chunk, that hash is

    keyed_hash(0^32, keyed_hash(DATA_KEY, content))       (printed as 4 little-endian u64s)

with DATA_KEY xet-core's public `merklehash` constant below.  A Xet chunk is at most 128 KiB,
so a single-chunk file pins a BLAKE3 tree of up to 128 chunks — more than any cas_id message
(le64(size) || content is at most 102,408 bytes = 101 chunks, cas.rs:23-62).  KEYED_HASH
mode shares the tree (chunk counters, parent merges, ROOT placement) with hash mode; only the
key words and flag 16 differ.

Selection is not circular: for each message length we draw contents until one hashes as a
single Xet chunk, i.e. until hf_xet's digest equals the oracle's.  A 256-bit match cannot be
accidental, so every recorded vector is an independent confirmation of the oracle's tree at
that length; a length with no single-chunk draw is listed under "unpinned", never dropped.
Content of a vector = numpy default_rng([len, seed]).integers(0, 256, len, uint8), with its
CRC-32 recorded to catch generator drift.
"""
import json
import os
import sys
import tempfile
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

DATA_KEY = bytes([102, 151, 245, 119, 91, 149, 80, 222, 49, 53, 203, 172, 165, 151, 24, 28,
                  157, 228, 33, 16, 155, 235, 43, 88, 180, 208, 176, 75, 147, 173, 242, 41])
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "xet_blake3.json")


def content(n: int, seed: int) -> bytes:
    return np.random.default_rng([n, seed]).integers(0, 256, n, dtype=np.uint8).tobytes()


def xet_display(digest: bytes) -> str:
    """MerkleHash's hex form: four u64 words, each printed as a big-endian hex number."""
    return "".join(digest[i:i + 8][::-1].hex() for i in range(0, 32, 8))


def single_chunk_xet(orc, data: bytes) -> str:
    return xet_display(orc.keyed_hash(bytes(32), orc.keyed_hash(DATA_KEY, data)))


def lengths():
    rng = np.random.default_rng(2026)
    out = {1, 63, 64, 65, 1023, 1024, 1025, 2048, 2049, 4096, 8 + 57_344, 8 + 102_400,
           8 + 102_399, 65_536, 131_071, 131_072}
    for c in range(1, 129):               # every chunk count 1..128, ragged last chunk
        out.add((c - 1) * 1024 + int(rng.integers(1, 1025)))
    return sorted(out)


def main():
    import hf_xet
    from importlib.metadata import version
    from oracle.pyoracle import Oracle
    orc = Oracle()
    vectors, unpinned = [], []
    with tempfile.TemporaryDirectory() as tmp:
        for n in lengths():
            hit = None
            for seed in range(0, 48, 8):      # draws in batches of 8 files per hf_xet call
                draws = [(s, content(n, s)) for s in range(seed, seed + 8)]
                paths = []
                for s, d in draws:
                    p = os.path.join(tmp, f"{n}_{s}.bin")
                    with open(p, "wb") as f:
                        f.write(d)
                    paths.append(p)
                for (s, d), r in zip(draws, hf_xet.hash_files(paths)):
                    if r.hash == single_chunk_xet(orc, d):
                        hit = {"len": n, "seed": s, "crc32": zlib.crc32(d), "xet_hash": r.hash}
                        break
                for p in paths:
                    os.unlink(p)
                if hit:
                    break
            (vectors.append(hit) if hit else unpinned.append(n))
    doc = {
        "source": f"hf_xet {version('hf_xet')} hash_files (Rust blake3 crate), single-Xet-chunk files",
        "relation": "xet_hash == hex4le64(keyed_hash(0^32, keyed_hash(DATA_KEY, content)))",
        "data_key": DATA_KEY.hex(),
        "content": "numpy default_rng([len, seed]).integers(0, 256, len, dtype=uint8)",
        "vectors": vectors,
        "unpinned": unpinned,
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=0)
        f.write("\n")
    print(f"{len(vectors)} vectors (max {max(v['len'] for v in vectors)} B), unpinned {unpinned}")


if __name__ == "__main__":
    main()
