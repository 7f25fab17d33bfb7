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
