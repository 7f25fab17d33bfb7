"""cas_id string consumers: thumbnail shard / key / path of a cas_id
(core/src/object/media/thumbnail/shard.rs:10-13, thumbnail/mod.rs:37-41,62-103).

CPU tests: the library's host functions (no GPU needed) against the oracle's restatement
(oracle/pyoracle.py: get_shard_hex, get_thumbnail_path with std's PathBuf::push /
set_extension rules, get_thumb_key).  The reference has no test for these functions, so
parity rests on the restatement plus the hand-written expectations below.
GPU test: the device batch formatters against the same oracle."""
import uuid

import numpy as np
import pytest

import spacedrive_amd as sd
from oracle.pyoracle import py_shard_hex, py_thumb_key, py_thumbnail_path
from spacedrive_amd import cas as sdcas

KEYS = [0, 1, 0xAF1349B9F5F9A1A6, 0xFFFFFFFFFFFFFFFF, 0x0123456789ABCDEF, 0xFFF0000000000000]
DIRS = ["/home/u/.local/share/spacedrive", "/data/", "/", "", "rel/dir", "/a b/ü"]
LIB = str(uuid.UUID("8c3c4fb3-7e2b-4d7e-9f0a-1b2c3d4e5f60"))


def test_hand_written_expectations():
    cas_id = "af1349b9f5f9a1a6"
    assert sdcas.get_shard_hex(cas_id) == "af1"
    assert sdcas.get_indexed_thumbnail_path("/srv/sd", cas_id, LIB) == \
        f"/srv/sd/thumbnails/{LIB}/af1/af1349b9f5f9a1a6.webp"
    assert sdcas.get_ephemeral_thumbnail_path("/srv/sd/", cas_id) == \
        "/srv/sd/thumbnails/ephemeral/af1/af1349b9f5f9a1a6.webp"
    assert sdcas.get_ephemeral_thumbnail_path("", cas_id) == "thumbnails/ephemeral/af1/af1349b9f5f9a1a6.webp"
    assert sdcas.get_indexed_thumb_key(cas_id, LIB) == [LIB, "af1", cas_id]
    assert sdcas.get_ephemeral_thumb_key(cas_id) == ["ephemeral", "af1", cas_id]
    assert sdcas.thumbnail_dir("/srv/sd", LIB) == f"/srv/sd/thumbnails/{LIB}/"


def test_host_functions_vs_oracle():
    rng = np.random.default_rng(5)
    keys = KEYS + [int(k) for k in rng.integers(0, 2 ** 63, 200, dtype=np.int64) * 2 + 1]
    for k in keys:
        cas_id = sdcas.key_to_cas_id(k)
        assert sdcas.get_shard_hex(cas_id) == py_shard_hex(cas_id)
        assert sdcas.get_ephemeral_thumb_key(cas_id) == py_thumb_key(cas_id)
        assert sdcas.get_indexed_thumb_key(cas_id, LIB) == py_thumb_key(cas_id, LIB)
        for d in DIRS:
            assert sdcas.get_ephemeral_thumbnail_path(d, cas_id) == py_thumbnail_path(d, cas_id)
            assert sdcas.get_indexed_thumbnail_path(d, cas_id, LIB) == py_thumbnail_path(d, cas_id, LIB)


def test_truncation_and_errors():
    import ctypes
    from spacedrive_amd import _native
    L = _native.lib()
    full = py_thumbnail_path("/srv/sd", "af1349b9f5f9a1a6", LIB)
    for cap in [1, 5, len(full), len(full) + 1, len(full) + 9]:
        buf = ctypes.create_string_buffer(b"\xff" * cap, cap)
        n = L.sd_cas_thumbnail_path(b"/srv/sd", LIB.encode(), 0xAF1349B9F5F9A1A6, buf, cap)
        assert n == len(full)  # snprintf-like: the full length whatever fits
        assert buf.raw[:cap].split(b"\0")[0].decode() == full[:cap - 1]
    assert L.sd_cas_thumbnail_path(None, None, 0, None, 0) == -1
    need = L.sd_cas_thumb_key(None, 0, None, 0)
    assert need == len("ephemeral") + 1 + 4 + 17
    with pytest.raises(ValueError):
        sdcas.get_shard_hex("af1")


@pytest.mark.gpu
def test_device_batches_vs_oracle(eng):
    import torch
    rng = np.random.default_rng(6)
    n = 100_003
    hk = rng.integers(0, 2 ** 64 - 1, n, dtype=np.uint64, endpoint=True)
    hk[:len(KEYS)] = np.array(KEYS, dtype=np.uint64)
    keys = torch.from_numpy(hk.view(np.int64)).cuda()
    hexes = torch.empty(16 * n, dtype=torch.uint8, device="cuda")
    eng.keys_to_hex(keys, hexes)
    got = hexes.cpu().numpy().tobytes()
    want = "".join(f"{int(k):016x}" for k in hk).encode()
    assert got == want
    idx = np.concatenate([np.arange(len(KEYS)), rng.choice(n, 2000, replace=False), [n - 1]])
    for data_dir, lib, stride in [("/srv/sd", None, 64), ("/home/u/.local/share/spacedrive", LIB, 128),
                                  ("", None, 48)]:
        prefix = sdcas.thumbnail_dir(data_dir, lib)
        out = torch.full((n * stride,), 0xAB, dtype=torch.uint8, device="cuda")
        eng.thumbnail_paths(keys, prefix, stride, out)
        rec = out.cpu().numpy().reshape(n, stride)
        for i in idx:
            path = py_thumbnail_path(data_dir, f"{int(hk[i]):016x}", lib).encode()
            assert rec[i, :len(path)].tobytes() == path, i
            assert not rec[i, len(path):].any(), i  # NUL padding
    with pytest.raises(sd.CasError):
        eng.thumbnail_paths(keys, "/srv/sd/thumbnails/ephemeral/", 32, out)
