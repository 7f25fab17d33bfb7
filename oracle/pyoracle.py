"""Python side of the oracle.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker / CPU baseline; nothing under spacedrive_amd/ does.

Two things live here:

* ``py_blake3`` — a third, pure-Python BLAKE3 restatement written independently of
  ``blake3_ref.c`` (recursive left-balanced tree, spec constants).  It is slow and used
  on small inputs to cross-check the C oracle.  The reference calls the external
  ``blake3`` 1.5.0 crate (reference ``Cargo.lock:1127-1139``) from
  ``core/src/object/cas.rs:24-61``.
* ``Oracle`` — ctypes bindings of ``oracle/liboracle_cas.so`` (built by
  ``oracle/Makefile``): the C restatement of ``generate_cas_id`` (``cas.rs:23-62``),
  ``file_checksum`` (``validation/hash.rs:11-25``), the grouping of
  ``file_identifier/mod.rs:98-350`` and the synthetic-content generator.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_cas.so")

# cas.rs:10-15
SAMPLE_COUNT = 4
SAMPLE_SIZE = 1024 * 10
HEADER_OR_FOOTER_SIZE = 1024 * 8
MINIMUM_FILE_SIZE = 1024 * 100
SAMPLED_CONTENT_LEN = 2 * HEADER_OR_FOOTER_SIZE + SAMPLE_COUNT * SAMPLE_SIZE  # 57,344
CHUNK_SIZE = 100  # file_identifier/mod.rs:34

# ---------------------------------------------------------------------------
# pure-Python BLAKE3 (independent restatement)
# ---------------------------------------------------------------------------
_IV = (0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
       0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19)
_PERM = (2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)
_M32 = 0xFFFFFFFF
CHUNK_START, CHUNK_END, PARENT, ROOT = 1, 2, 4, 8
DERIVE_KEY_CONTEXT, DERIVE_KEY_MATERIAL = 32, 64
KEYED_HASH = 16


def _rotr(x: int, n: int) -> int:
    return ((x >> n) | (x << (32 - n))) & _M32


def _compress(cv, block: bytes, counter: int, blen: int, flags: int):
    m = [int.from_bytes(block[4 * i:4 * i + 4], "little") for i in range(16)]
    v = list(cv) + list(_IV[:4]) + [counter & _M32, (counter >> 32) & _M32, blen, flags]

    def g(a, b, c, d, x, y):
        v[a] = (v[a] + v[b] + x) & _M32
        v[d] = _rotr(v[d] ^ v[a], 16)
        v[c] = (v[c] + v[d]) & _M32
        v[b] = _rotr(v[b] ^ v[c], 12)
        v[a] = (v[a] + v[b] + y) & _M32
        v[d] = _rotr(v[d] ^ v[a], 8)
        v[c] = (v[c] + v[d]) & _M32
        v[b] = _rotr(v[b] ^ v[c], 7)

    for r in range(7):
        g(0, 4, 8, 12, m[0], m[1]); g(1, 5, 9, 13, m[2], m[3])
        g(2, 6, 10, 14, m[4], m[5]); g(3, 7, 11, 15, m[6], m[7])
        g(0, 5, 10, 15, m[8], m[9]); g(1, 6, 11, 12, m[10], m[11])
        g(2, 7, 8, 13, m[12], m[13]); g(3, 4, 9, 14, m[14], m[15])
        m = [m[p] for p in _PERM]
    return [v[i] ^ v[i + 8] for i in range(8)] + [v[i + 8] ^ cv[i] for i in range(8)]


def _chunk_node(key, data: bytes, counter: int, flags: int):
    """Returns (cv_in, last_block, blen, counter, flags) of the chunk's final block."""
    cv = list(key)
    blocks = [data[i:i + 64] for i in range(0, len(data), 64)] or [b""]
    for i, blk in enumerate(blocks):
        f = flags | (CHUNK_START if i == 0 else 0) | (CHUNK_END if i == len(blocks) - 1 else 0)
        padded = blk + bytes(64 - len(blk))
        if i == len(blocks) - 1:
            return (cv, padded, len(blk), counter, f)
        cv = _compress(cv, padded, counter, 64, f)[:8]
    raise AssertionError


def _node_cv(node):
    cv, blk, blen, ctr, f = node
    return _compress(cv, blk, ctr, blen, f)[:8]


def _subtree(key, data: bytes, chunk0: int, flags: int):
    if len(data) <= 1024:
        return _chunk_node(key, data, chunk0, flags)
    n = (len(data) + 1023) // 1024
    left = 1
    while left * 2 < n:
        left *= 2
    lcv = _node_cv(_subtree(key, data[:left * 1024], chunk0, flags))
    rcv = _node_cv(_subtree(key, data[left * 1024:], chunk0 + left, flags))
    blk = b"".join(w.to_bytes(4, "little") for w in lcv + rcv)
    return (list(key), blk, 64, 0, flags | PARENT)


def _root_bytes(node, out_len=32) -> bytes:
    cv, blk, blen, _ctr, f = node
    w = _compress(cv, blk, 0, blen, f | ROOT)
    return b"".join(x.to_bytes(4, "little") for x in w)[:out_len]


def py_blake3(data: bytes, out_len: int = 32) -> bytes:
    return _root_bytes(_subtree(_IV, bytes(data), 0, 0), out_len)


def py_derive_key(context: str, material: bytes) -> bytes:
    ck = _root_bytes(_subtree(_IV, context.encode(), 0, DERIVE_KEY_CONTEXT))
    key = [int.from_bytes(ck[4 * i:4 * i + 4], "little") for i in range(8)]
    return _root_bytes(_subtree(key, bytes(material), 0, DERIVE_KEY_MATERIAL))


def py_keyed_hash(key: bytes, data: bytes) -> bytes:
    """blake3::keyed_hash: the 32-byte key replaces IV, KEYED_HASH on every compression."""
    k = [int.from_bytes(key[4 * i:4 * i + 4], "little") for i in range(8)]
    return _root_bytes(_subtree(k, bytes(data), 0, KEYED_HASH))


def py_sample_plan(size: int):
    """cas.rs:35-58 simulated literally: [(offset, length)] x 6, for a file whose actual
    length is `size` (the footer is SeekFrom::End(-8192), i.e. relative to the actual end;
    py_generate_cas_id_file covers files whose length differs from their metadata)."""
    H, S = HEADER_OR_FOOTER_SIZE, SAMPLE_SIZE
    plan = [(0, H)]
    cursor = H
    current_pos = H
    seek_jump = (size - H * 2) // SAMPLE_COUNT
    while True:
        plan.append((cursor, S))
        cursor += S
        if current_pos >= H + seek_jump * (SAMPLE_COUNT - 1):
            break
        current_pos = current_pos + seek_jump
        cursor = current_pos
    plan.append((size - H, H))
    return plan


class UnexpectedEof(OSError):
    """tokio read_exact's io::ErrorKind::UnexpectedEof (mapped to EIO by the C ABI)."""


def py_generate_cas_id_file(path: str, size: int) -> str:
    """cas.rs:23-62 executed literally on a real file with the same sequence of reads and
    seeks (read_exact = read until full or EOF; seek(Start), seek(End(-8192))).  Unlike
    py_sample_plan this follows the file's ACTUAL length for the footer, as the reference
    does when the file changed after fs::metadata."""
    H, S = HEADER_OR_FOOTER_SIZE, SAMPLE_SIZE
    parts = [int(size).to_bytes(8, "little")]
    if size <= MINIMUM_FILE_SIZE:
        with open(path, "rb") as fh:  # fs::read: the whole file as it is now
            parts.append(fh.read())
        return py_blake3(b"".join(parts)).hex()[:16]

    def read_exact(fh, n):
        b = b""
        while len(b) < n:
            x = fh.read(n - len(b))
            if not x:
                raise UnexpectedEof(5, "failed to fill whole buffer")
            b += x
        return b

    with open(path, "rb") as fh:
        parts.append(read_exact(fh, H))
        current_pos = H
        seek_jump = (size - H * 2) // SAMPLE_COUNT
        while True:
            parts.append(read_exact(fh, S))
            if current_pos >= H + seek_jump * (SAMPLE_COUNT - 1):
                break
            current_pos = fh.seek(current_pos + seek_jump, os.SEEK_SET)
        end = os.fstat(fh.fileno()).st_size
        if end < H:
            raise OSError(22, "invalid seek to a negative or overflowing position")
        fh.seek(-H, os.SEEK_END)
        parts.append(read_exact(fh, H))
    return py_blake3(b"".join(parts)).hex()[:16]


def py_cas_message(content: bytes, size: int) -> bytes:
    return int(size).to_bytes(8, "little") + bytes(content)


def py_cas_id(content: bytes, size: int) -> str:
    """generate_cas_id on already-gathered content (cas.rs:24-61)."""
    return py_blake3(py_cas_message(content, size)).hex()[:16]


# ---------------------------------------------------------------------------
# cas_id string consumers: thumbnails (core/src/object/media/thumbnail/)
# ---------------------------------------------------------------------------
THUMBNAIL_CACHE_DIR_NAME = "thumbnails"  # mod.rs:37
WEBP_EXTENSION = "webp"                  # mod.rs:40
EPHEMERAL_DIR = "ephemeral"              # mod.rs:41


def py_shard_hex(cas_id: str) -> str:
    """get_shard_hex (shard.rs:10-13): &cas_id[0..3]."""
    return cas_id[0:3]


def _pathbuf_push(base: str, comp: str) -> str:
    """std PathBuf::push on Unix: an absolute component replaces the path; otherwise one '/'
    separates the components unless the base is empty or already ends in '/'."""
    if comp.startswith("/"):
        return comp
    if not base:
        return comp
    return base + ("" if base.endswith("/") else "/") + comp


def _pathbuf_set_extension(path: str, ext: str) -> str:
    """std PathBuf::set_extension: replace the file name's extension (the part after its
    last '.', a leading '.' of a dot-file not counting) with `ext`."""
    d, sep, name = path.rpartition("/")
    stem = name
    i = name.rfind(".")
    if i > 0:
        stem = name[:i]
    name = stem + ("." + ext if ext else "")
    return d + sep + name


def py_thumbnail_path(data_dir: str, cas_id: str, library_id=None) -> str:
    """get_thumbnail_path (mod.rs:67-82); library_id None = ThumbnailKind::Ephemeral."""
    p = _pathbuf_push(data_dir, THUMBNAIL_CACHE_DIR_NAME)
    p = _pathbuf_push(p, EPHEMERAL_DIR if library_id is None else str(library_id))
    p = _pathbuf_push(p, py_shard_hex(cas_id))
    p = _pathbuf_push(p, cas_id)
    return _pathbuf_set_extension(p, WEBP_EXTENSION)


def py_thumb_key(cas_id: str, library_id=None) -> list:
    """get_thumb_key (mod.rs:94-103)."""
    return [EPHEMERAL_DIR if library_id is None else str(library_id), py_shard_hex(cas_id), cas_id]


# ---------------------------------------------------------------------------
# synthetic content (same counter-based splitmix64 as oracle/cas_ref.c and the device)
# ---------------------------------------------------------------------------
_G = np.uint64(0x9E3779B97F4A7C15)


def np_mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def np_file_key(seed: int, files):
    with np.errstate(over="ignore"):
        return np_mix64(np_mix64(np.uint64(seed)) + np.asarray(files, dtype=np.uint64) * _G)


def np_content(seed: int, file: int, length: int) -> bytes:
    key = np_file_key(seed, file)
    nw = (length + 7) // 8
    with np.errstate(over="ignore"):
        w = np_mix64(key + (np.arange(1, nw + 1, dtype=np.uint64) * _G))
    return w.astype("<u8").tobytes()[:length]


# ---------------------------------------------------------------------------
# ctypes bindings of the C oracle
# ---------------------------------------------------------------------------
def build_oracle(quiet: bool = True) -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)
    return LIB_PATH


EXT_PATH = os.path.join(HERE, "libext_b3.so")


class ExtBlake3:
    """The BLAKE3 team's C implementation (1.8.2, dlopened from ROCm's libclang-cpp.so by
    oracle/ext_b3.c) run through cas.rs's per-file call sequence — bench.py's second CPU
    baseline leg and a parity check; never the product."""

    def __init__(self, path: str = EXT_PATH):
        if not os.path.exists(path):
            build_oracle()
        L = ctypes.CDLL(path)
        L.ext_b3_load.restype = ctypes.c_int
        L.ext_b3_version.restype = ctypes.c_char_p
        L.ext_b3_cas_keys_strided.restype = ctypes.c_int
        L.ext_b3_cas_keys_strided.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                              ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                              ctypes.c_int]
        L.ext_b3_file_checksum.restype = ctypes.c_int
        L.ext_b3_file_checksum.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.ext_b3_file_checksums.restype = ctypes.c_int
        L.ext_b3_file_checksums.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p]
        L.ext_b3_cas_keys_paths.restype = ctypes.c_int
        L.ext_b3_cas_keys_paths.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        if L.ext_b3_load() != 0:
            raise OSError("libclang-cpp.so with the BLAKE3 C API not found")
        self.L = L

    def version(self) -> str:
        return self.L.ext_b3_version().decode()

    def file_checksum(self, path: str) -> str:
        """hash.rs:11-25 streamed (1 MiB reads, one hasher) through the C library."""
        out = ctypes.create_string_buffer(65)
        rc = self.L.ext_b3_file_checksum(os.fsencode(path), out)
        if rc != 0:
            raise OSError(-rc, os.strerror(-rc) if rc > -1000 else "no library", path)
        return out.value.decode()

    def file_checksums(self, paths, threads: int = 1):
        """(hex digest or None, -errno) per path, files interleaved over `threads`."""
        n = len(paths)
        keep = [os.fsencode(p) for p in paths]
        parr = (ctypes.c_char_p * max(n, 1))(*keep)
        hexbuf = ctypes.create_string_buffer(65 * max(n, 1))
        status = np.zeros(n, dtype=np.int32)
        if self.L.ext_b3_file_checksums(ctypes.cast(parr, ctypes.c_void_p), n, int(threads), hexbuf,
                                        status.ctypes.data) != 0:
            raise OSError("ext_b3_file_checksums failed")
        raw = hexbuf.raw
        return [None if status[i] else raw[65 * i:65 * i + 64].decode() for i in range(n)], -status

    def cas_keys_paths(self, paths, sizes, threads: int = 1):
        """(keys u64, status -errno): cas.rs's reads, then the C library's hashing."""
        n = len(paths)
        keep = [os.fsencode(p) for p in paths]
        parr = (ctypes.c_char_p * max(n, 1))(*keep)
        sz = _sizes_u64(sizes)
        keys = np.zeros(n, dtype=np.uint64)
        status = np.zeros(n, dtype=np.int32)
        if self.L.ext_b3_cas_keys_paths(ctypes.cast(parr, ctypes.c_void_p), sz.ctypes.data, n,
                                        int(threads), keys.ctypes.data, status.ctypes.data) != 0:
            raise OSError("ext_b3_cas_keys_paths failed")
        return keys, status

    def cas_keys_strided(self, arena: np.ndarray, stride: int, clen: int, sizes,
                         threads: int = 1) -> np.ndarray:
        sz = _sizes_u64(sizes)
        n = len(sz)
        a = np.ascontiguousarray(arena, dtype=np.uint8)
        assert n == 0 or a.size >= (n - 1) * stride + clen
        out = np.zeros(n, dtype=np.uint64)
        rc = self.L.ext_b3_cas_keys_strided(a.ctypes.data, stride, clen, sz.ctypes.data, n,
                                            out.ctypes.data, threads)
        if rc != 0:
            raise OSError("ext_b3_cas_keys_strided failed")
        return out


def _sizes_u64(sizes) -> np.ndarray:
    """Sizes as u64; a negative entry of a signed array is refused instead of wrapping to
    2^64 - 1 (the same check as the product wrapper's, spacedrive_amd/cas.py)."""
    a = np.asarray(sizes)
    if a.size and a.dtype.kind == "i" and int(a.min()) < 0:
        raise ValueError(f"negative size {int(a.min())}")
    return np.ascontiguousarray(a, dtype=np.uint64)


class Oracle:
    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            build_oracle()
        L = ctypes.CDLL(path)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        sz = ctypes.c_size_t
        L.orc_blake3.argtypes = [ctypes.c_void_p, sz, ctypes.c_void_p, sz]
        L.orc_blake3_recursive.argtypes = [ctypes.c_void_p, sz, ctypes.c_void_p]
        L.orc_blake3_levelwise.argtypes = [ctypes.c_void_p, sz, ctypes.c_void_p]
        L.orc_blake3_derive_key.argtypes = [ctypes.c_char_p, ctypes.c_void_p, sz, ctypes.c_void_p]
        L.orc_blake3_keyed.argtypes = [ctypes.c_char_p, ctypes.c_void_p, sz, ctypes.c_void_p]
        L.orc_sample_plan.argtypes = [ctypes.c_uint64, u64p, u64p]
        L.orc_cas_key.argtypes = [ctypes.c_void_p, sz, ctypes.c_uint64]
        L.orc_cas_key.restype = ctypes.c_uint64
        L.orc_cas_keys.argtypes = [ctypes.c_void_p, u64p, u64p, u64p, sz, u64p, ctypes.c_int]
        L.orc_cas_keys_strided.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                           u64p, sz, u64p, ctypes.c_int]
        L.orc_fast_cas_keys.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_uint64, ctypes.c_uint64, u64p, sz, u64p,
                                        ctypes.c_int]
        L.orc_fast_has_simd.restype = ctypes.c_int
        L.orc_generate_cas_id.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        L.orc_generate_cas_id.restype = ctypes.c_int
        L.orc_generate_cas_keys_paths.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_generate_cas_keys_paths.restype = None
        L.orc_fast_generate_cas_keys_paths.argtypes = L.orc_generate_cas_keys_paths.argtypes
        L.orc_fast_generate_cas_keys_paths.restype = None
        L.orc_file_checksum.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_file_checksum.restype = ctypes.c_int
        L.orc_blake3_mt.argtypes = [ctypes.c_void_p, sz, ctypes.c_int, ctypes.c_void_p]
        L.orc_stream_blake3_mt.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_int, ctypes.c_void_p]
        L.orc_file_checksum_mt.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
        L.orc_file_checksum_mt.restype = ctypes.c_int
        L.orc_fill_content_range.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_void_p, sz]
        L.orc_gather_path.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p, sz]
        L.orc_gather_path.restype = ctypes.c_int64
        L.orc_group_canonical.argtypes = [u64p, sz, u32p]
        L.orc_group_canonical.restype = ctypes.c_uint64
        L.orc_group_chunked.argtypes = [u64p, sz, sz, u32p, u64p, u64p]
        L.orc_fill_content.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, sz]
        L.orc_synth_root.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.orc_synth_root.restype = ctypes.c_uint64
        L.orc_synth_size.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.orc_synth_size.restype = ctypes.c_uint64
        L.orc_balloon_blake3.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.c_char_p,
                                         sz, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p]
        L.orc_balloon_blake3.restype = ctypes.c_int
        self.L = L
        _ = u8p

    # -- BLAKE3 --------------------------------------------------------------
    def blake3(self, data: bytes, out_len: int = 32) -> bytes:
        out = ctypes.create_string_buffer(out_len)
        self.L.orc_blake3(data, len(data), out, out_len)
        return out.raw

    def blake3_recursive(self, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.L.orc_blake3_recursive(data, len(data), out)
        return out.raw

    def blake3_levelwise(self, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.L.orc_blake3_levelwise(data, len(data), out)
        return out.raw

    def blake3_mt(self, data, threads: int = 8) -> bytes:
        """Tree-parallel BLAKE3 (16 MiB subtrees); data: bytes or a contiguous uint8 array."""
        out = ctypes.create_string_buffer(32)
        if isinstance(data, np.ndarray):
            self.L.orc_blake3_mt(data.ctypes.data, data.nbytes, threads, out)
        else:
            self.L.orc_blake3_mt(data, len(data), threads, out)
        return out.raw

    def stream_blake3_mt(self, seed: int, file: int, length: int, threads: int = 8) -> bytes:
        """BLAKE3 of the first `length` bytes of the synthetic stream of (seed, file)."""
        out = ctypes.create_string_buffer(32)
        self.L.orc_stream_blake3_mt(seed, file, length, threads, out)
        return out.raw

    def fill_content_range(self, seed: int, file: int, off: int, length: int) -> np.ndarray:
        out = np.empty(max(length, 1), dtype=np.uint8)
        self.L.orc_fill_content_range(seed, file, off, out.ctypes.data, length)
        return out[:length]

    def file_checksum_mt(self, path: str, threads: int = 8) -> str:
        out = ctypes.create_string_buffer(65)
        rc = self.L.orc_file_checksum_mt(path.encode(), threads, out)
        if rc != 0:
            raise OSError(-rc, os.strerror(-rc), path)
        return out.value.decode()

    def keyed_hash(self, key: bytes, data: bytes) -> bytes:
        assert len(key) == 32
        out = ctypes.create_string_buffer(32)
        self.L.orc_blake3_keyed(key, data, len(data), out)
        return out.raw

    def derive_key(self, context: str, material: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.L.orc_blake3_derive_key(context.encode(), material, len(material), out)
        return out.raw

    def balloon_blake3(self, password: bytes, salt: bytes, secret: bytes | None, s_cost: int,
                       t_cost: int) -> bytes:
        """Balloon::<blake3::Hasher> (balloon_ref.c), the reference's password hash
        (crates/crypto/src/keys/hashing.rs:95-114): its KATs pin multi-block BLAKE3."""
        out = ctypes.create_string_buffer(32)
        rc = self.L.orc_balloon_blake3(password, len(password), salt, len(salt), secret,
                                       len(secret or b""), s_cost, t_cost, out)
        if rc:
            raise ValueError("balloon: bad sizes")
        return out.raw

    # -- cas -----------------------------------------------------------------
    def sample_plan(self, size: int):
        o = (ctypes.c_uint64 * 6)()
        ln = (ctypes.c_uint64 * 6)()
        self.L.orc_sample_plan(size, o, ln)
        return [(o[i], ln[i]) for i in range(6)]

    def cas_key(self, content: bytes, size: int) -> int:
        return int(self.L.orc_cas_key(content, len(content), size))

    def cas_id(self, content: bytes, size: int) -> str:
        return f"{self.cas_key(content, size):016x}"

    def cas_keys(self, arena: np.ndarray, offs: np.ndarray, lens: np.ndarray,
                 sizes: np.ndarray, threads: int = 1) -> np.ndarray:
        n = len(sizes)
        out = np.zeros(n, dtype=np.uint64)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        sizes = _sizes_u64(sizes)
        self.L.orc_cas_keys(arena.ctypes.data, _p64(offs), _p64(lens), _p64(sizes), n,
                            _p64(out), threads)
        return out

    def cas_keys_strided(self, arena: np.ndarray, stride: int, clen: int, sizes: np.ndarray,
                         threads: int = 1) -> np.ndarray:
        n = len(sizes)
        out = np.zeros(n, dtype=np.uint64)
        sizes = _sizes_u64(sizes)
        self.L.orc_cas_keys_strided(arena.ctypes.data, stride, clen, _p64(sizes), n, _p64(out),
                                    threads)
        return out

    def fast_cas_keys_strided(self, arena: np.ndarray, stride: int, clen: int,
                              sizes: np.ndarray, threads: int = 1) -> np.ndarray:
        n = len(sizes)
        out = np.zeros(n, dtype=np.uint64)
        sizes = _sizes_u64(sizes)
        self.L.orc_fast_cas_keys(arena.ctypes.data, None, None, stride, clen, _p64(sizes), n,
                                 _p64(out), threads)
        return out

    def fast_cas_keys(self, arena: np.ndarray, offs, lens, sizes, threads: int = 1) -> np.ndarray:
        n = len(sizes)
        out = np.zeros(n, dtype=np.uint64)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        sizes = _sizes_u64(sizes)
        self.L.orc_fast_cas_keys(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, 0, 0,
                                 _p64(sizes), n, _p64(out), threads)
        return out

    def has_simd(self) -> bool:
        return bool(self.L.orc_fast_has_simd())

    def generate_cas_id(self, path: str, size: int) -> str:
        out = ctypes.create_string_buffer(17)
        rc = self.L.orc_generate_cas_id(path.encode(), size, out)
        if rc != 0:
            raise OSError(-rc, os.strerror(-rc), path)
        return out.value.decode()

    def generate_cas_keys_paths(self, paths, sizes, threads: int = 1, simd: bool = False):
        """(keys u64, status -errno) for many paths, files interleaved over `threads`;
        simd=True hashes sampled files 16 at a time with the AVX-512 baseline."""
        n = len(paths)
        # one joined buffer for ASCII str paths (the marshalling cost the product's wrapper
        # pays too, so per-step timings of the two compare like for like)
        joined = "\0".join(paths) + "\0" if n and all(type(p) is str for p in paths) else None
        buf = os.fsencode(joined) if joined is not None else None
        if buf is not None and len(buf) == len(joined) and joined.count("\0") == n:
            cbuf = ctypes.c_char_p(buf)
            lens = np.fromiter(map(len, paths), dtype=np.uint64, count=n) + np.uint64(1)
            ptrs = np.zeros(n, dtype=np.uint64)
            np.cumsum(lens[:-1], out=ptrs[1:])
            ptrs += np.uint64(ctypes.cast(cbuf, ctypes.c_void_p).value)
            parr_addr = ptrs.ctypes.data
        else:
            parr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
            parr_addr = ctypes.cast(parr, ctypes.c_void_p).value
        sz = _sizes_u64(sizes)
        keys = np.zeros(n, dtype=np.uint64)
        status = np.zeros(n, dtype=np.int32)
        fn = self.L.orc_fast_generate_cas_keys_paths if simd else self.L.orc_generate_cas_keys_paths
        fn(parr_addr, sz.ctypes.data, n, int(threads), keys.ctypes.data, status.ctypes.data)
        return keys, status

    def file_checksum(self, path: str) -> str:
        out = ctypes.create_string_buffer(65)
        rc = self.L.orc_file_checksum(path.encode(), out)
        if rc != 0:
            raise OSError(-rc, os.strerror(-rc), path)
        return out.value.decode()

    def gather_path(self, path: str, size: int, cap: int = MINIMUM_FILE_SIZE + 1) -> bytes:
        cap = max(cap, SAMPLED_CONTENT_LEN)
        buf = ctypes.create_string_buffer(cap)
        n = self.L.orc_gather_path(path.encode(), size, buf, cap)
        if n < 0:
            raise OSError(-n, os.strerror(-n), path)
        return buf.raw[:n]

    # -- grouping ------------------------------------------------------------
    def group_canonical(self, keys: np.ndarray):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        rep = np.zeros(len(keys), dtype=np.uint32)
        objects = self.L.orc_group_canonical(_p64(keys), len(keys), _p32(rep))
        return rep, int(objects)

    def group_chunked(self, keys: np.ndarray, chunk: int = CHUNK_SIZE):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        rep = np.zeros(len(keys), dtype=np.uint32)
        c = ctypes.c_uint64()
        ln = ctypes.c_uint64()
        self.L.orc_group_chunked(_p64(keys), len(keys), chunk, _p32(rep), ctypes.byref(c),
                                 ctypes.byref(ln))
        return rep, int(c.value), int(ln.value)

    def synth_root(self, seed: int, file: int, dup_permille: int) -> int:
        return int(self.L.orc_synth_root(seed, file, dup_permille))

    def synth_size(self, seed: int, root: int, kind: int) -> int:
        return int(self.L.orc_synth_size(seed, root, kind))

    def fill_content(self, seed: int, file: int, length: int) -> bytes:
        buf = ctypes.create_string_buffer(max(length, 1))
        self.L.orc_fill_content(seed, file, buf, length)
        return buf.raw[:length]


def _p64(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def _p32(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
