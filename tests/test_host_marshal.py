"""Host-side marshalling of the batch path calls (spacedrive_amd.cas._path_array): the
`const char* const* paths` array the C ABI reads must hold every path's bytes exactly as
os.fsencode gives them, for the fast joined-buffer case and the per-path fallback."""
import ctypes
import os
import pathlib

import numpy as np

from spacedrive_amd.cas import _path_array


def _read_back(paths):
    keep, addr = _path_array(paths)
    arr = (ctypes.c_char_p * max(len(paths), 1)).from_address(addr)
    out = [arr[i] for i in range(len(paths))]
    del keep
    return out


def test_ascii_paths_joined():
    paths = [f"/dev/shm/dir{i % 7}/file_{i:05d}.bin" for i in range(257)] + ["a", "/"]
    assert _read_back(paths) == [os.fsencode(p) for p in paths]


def test_fallbacks_non_ascii_bytes_pathlike():
    for paths in (["/tmp/é", "/tmp/a", "/tmp/日本"],
                  [b"/tmp/raw\xff", b"/tmp/b"],
                  [pathlib.Path("/tmp/p1"), "/tmp/p2"],
                  ["/tmp/bad\udcff", "/tmp/ok"]):
        assert _read_back(paths) == [os.fsencode(p) for p in paths]


def test_empty_and_single():
    assert _read_back([]) == []
    assert _read_back(["x"]) == [b"x"]


def test_keepalive_holds_pointer_targets():
    paths = [f"/p/{i}" for i in range(100)]
    keep, addr = _path_array(paths)
    ptrs = np.frombuffer((ctypes.c_uint64 * 100).from_address(addr), dtype=np.uint64)
    assert all(ctypes.string_at(int(p)) == os.fsencode(s) for p, s in zip(ptrs, paths))
    assert keep is not None


def test_sizes_and_object_ids_refused_before_the_abi():
    """a negative size of a signed array must not wrap to 2^64 - 1 (it would be
    gathered as a huge sampled file), and Object ids outside [0, 2^31) must not reach the
    link emission (bit 31 is the seeded grouping's row tag) — both checked host-side."""
    import numpy as np
    import pytest
    from oracle.pyoracle import _sizes_u64 as orc_sizes
    from spacedrive_amd.cas import NO_OBJECT, _object_ids, _sizes_u64
    assert _sizes_u64(np.array([0, 5, 2 ** 40], np.int64)).dtype == np.uint64
    assert list(_sizes_u64([1, 2])) == [1, 2]
    for f in (_sizes_u64, orc_sizes):
        with pytest.raises(ValueError):
            f(np.array([10, -1], np.int64))
    assert list(_sizes_u64(np.array([2 ** 64 - 1], np.uint64))) == [2 ** 64 - 1]  # unsigned: as given
    assert list(_object_ids([3, None, -1, 2 ** 31 - 1], "x", none_ok=True)) == [3, NO_OBJECT, NO_OBJECT, 2 ** 31 - 1]
    for bad in ([2 ** 31], [-2], np.array([2 ** 31], np.uint32)):
        with pytest.raises(ValueError):
            _object_ids(bad, "x", none_ok=True)
    with pytest.raises(ValueError):
        _object_ids([-1], "x", none_ok=False)
