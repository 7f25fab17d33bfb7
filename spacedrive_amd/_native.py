"""ctypes binding of libsd_hip_cas.so (C ABI: include/sd_hip_cas.h).

The product path: every digest comes from the gfx950 kernels behind this library.
There is no CPU fallback — if the library is missing, or no gfx950 device is present,
the calls raise.  ``build()`` compiles it in-tree with hipcc (spacedrive_amd/csrc/Makefile).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
# SD_HIP_CAS_LIB lets profiling tools A/B two builds of the same library; default in-tree.
LIB_PATH = os.environ.get("SD_HIP_CAS_LIB") or os.path.join(HERE, "libsd_hip_cas.so")
CSRC = os.path.join(HERE, "csrc")

SD_CAS_OK = 0
ERRORS = {-1: "EINVAL", -2: "EHIP", -3: "EIO", -4: "ENOMEM", -5: "ENODEV"}

# (name, restype, argtypes) for every symbol declared in include/sd_hip_cas.h
_vp, _sz, _u64, _u32, _i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
_cp = ctypes.c_char_p
SIGNATURES = [
    ("sd_cas_abi_version", _i, []),
    ("sd_cas_ctx_create", _i, [_i, ctypes.POINTER(_vp)]),
    ("sd_cas_ctx_destroy", None, [_vp]),
    ("sd_cas_last_error", _cp, [_vp]),
    ("sd_cas_ctx_stream", _vp, [_vp]),
    ("sd_cas_synchronize", _i, [_vp]),
    ("sd_cas_batch_quantum", _sz, [_vp]),
    ("sd_cas_set_latency_threshold", None, [_vp, _sz, _sz]),
    ("sd_cas_set_chunkpar_split", None, [_vp, _sz, _sz]),
    ("sd_cas_set_group_method", _i, [_vp, _i, _u64]),
    ("sd_cas_alloc_pinned", _i, [_vp, _sz, ctypes.POINTER(_vp)]),
    ("sd_cas_free_pinned", _i, [_vp, _vp]),
    ("sd_cas_generate_cas_ids", _i, [_vp, _vp, _vp, _vp, _sz, _vp]),
    ("sd_cas_generate_cas_ids_from_paths", _i, [_vp, _vp, _vp, _sz, _vp, _vp]),
    ("sd_cas_file_metadata_from_paths", _i, [_vp, _vp, _sz, _vp, _vp, _vp]),
    ("sd_cas_hash_sampled_host", _i, [_vp, _vp, _u64, _vp, _sz, _vp, _sz]),
    ("sd_cas_hash_sampled_host_ring", _i, [_vp, _vp, _u64, _sz, _vp, _sz, _vp, _sz]),
    ("sd_cas_key_to_hex", None, [_u64, _cp]),
    ("sd_cas_shard_hex", None, [_u64, _cp]),
    ("sd_cas_thumbnail_path", ctypes.c_int64, [_cp, _cp, _u64, _cp, _sz]),
    ("sd_cas_thumb_key", ctypes.c_int64, [_cp, _u64, _cp, _sz]),
    ("sd_cas_keys_to_hex_dev", _i, [_vp, _vp, _sz, _vp, _vp]),
    ("sd_cas_thumbnail_paths_dev", _i, [_vp, _vp, _sz, _cp, _u32, _vp, _vp]),
    ("sd_cas_hash_sampled_dev", _i, [_vp, _vp, _u64, _vp, _sz, _vp, _vp]),
    ("sd_cas_hash_packed_dev", _i, [_vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    ("sd_cas_group_dev", _i, [_vp, _vp, _sz, _vp, _vp, _vp]),
    ("sd_cas_hash_group_sampled_dev", _i, [_vp, _vp, _u64, _vp, _sz, _vp, _vp, _vp, _vp, _vp]),
    ("sd_cas_hash_regions_sampled_dev", _i, [_vp, _vp, _u64, _vp, _sz, _vp, _vp, _vp, _vp]),
    ("sd_cas_group_regions_dev", _i, [_vp, _sz, _vp, _vp, _vp]),
    ("sd_cas_group_min_dev", _i, [_vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    ("sd_cas_partition_dev", _i, [_vp, _vp, _sz, _u32, _vp, _vp, _vp, _vp]),
    ("sd_cas_exchange_pack_dev", _i, [_vp, _vp, _vp, _sz, _u64, _vp, _vp]),
    ("sd_cas_exchange_split_dev", _i, [_vp, _vp, _sz, _vp, _vp, _vp]),
    ("sd_cas_exchange_unpack_dev", _i, [_vp, _vp, _vp, _sz, _vp, _vp]),
    ("sd_cas_exchange_pack_fixed_dev", _i, [_vp, _vp, _vp, _vp, _u32, _u64, _u64, _u64, _vp, _vp, _vp, _vp]),
    ("sd_cas_exchange_split_fixed_dev", _i, [_vp, _vp, _sz, _u64, _vp, _vp, _vp, _vp]),
    ("sd_cas_exchange_unpack_fixed_dev", _i, [_vp, _vp, _vp, _vp, _vp, _u32, _u64, _u64, _vp, _vp]),
    ("sd_cas_copy_objects_dev", _i, [_vp, _vp, _vp]),
    ("sd_cas_group_sorted_dev", _i, [_vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    ("sd_cas_group_chunked_dev", _i, [_vp, _vp, _sz, _u32, _vp, _vp, _vp, _vp]),
    ("sd_cas_identifier_max_steps", _sz, [_sz, _u32]),
    ("sd_cas_identifier_links_dev", _i, [_vp, _vp, _vp, _sz, _u32, _vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    ("sd_cas_identifier_links", _i, [_vp, _vp, _vp, _sz, _u32, _vp, _vp, _vp, _vp, _sz, _vp]),
    ("sd_cas_identifier_links_seeded_dev", _i,
     [_vp, _vp, _vp, _sz, _u32, _vp, _vp, _sz, _vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    ("sd_cas_identifier_links_seeded", _i,
     [_vp, _vp, _vp, _sz, _u32, _vp, _vp, _sz, _vp, _vp, _vp, _vp, _sz, _vp]),
    ("sd_cas_identifier_links_ex_dev", _i,
     [_vp, _vp, _vp, _sz, _u32, _vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    ("sd_cas_identifier_links_ex", _i,
     [_vp, _vp, _vp, _sz, _u32, _vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    ("sd_cas_sort_pairs_dev", _i, [_vp, _vp, _vp, _sz, _vp, _vp, _i, _i, _vp]),
    ("sd_cas_checksum_dev", _i, [_vp, _vp, _u64, _vp, _vp]),
    ("sd_cas_file_checksum", _i, [_vp, _cp, _cp, ctypes.POINTER(_i)]),
    ("sd_cas_checksums_dev", _i, [_vp, _vp, _u64, _vp, _vp, _sz, _vp, _vp]),
    ("sd_cas_file_checksums", _i, [_vp, _vp, _sz, _vp, _vp]),
    ("sd_cas_multi_create", _i, [_vp, _i, ctypes.POINTER(_vp)]),
    ("sd_cas_multi_destroy", None, [_vp]),
    ("sd_cas_multi_count", _i, [_vp]),
    ("sd_cas_multi_ctx", _vp, [_vp, _i]),
    ("sd_cas_multi_last_error", _cp, [_vp]),
    ("sd_cas_multi_group", _i, [_vp, _vp, _vp, _vp, _vp, _vp]),
    ("sd_cas_multi_hash_group_sampled_host", _i, [_vp, _vp, _u64, _vp, _sz, _vp, _vp, _vp]),
    ("sd_cas_synth_sampled_dev", _i, [_vp, _u64, _u64, _sz, _u32, _vp, _u64, _vp, _vp]),
    ("sd_cas_synth_small_dev", _i, [_vp, _u64, _u64, _sz, _u32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("sd_cas_synth_small_content_dev", _i, [_vp, _u64, _u64, _sz, _u32, _vp, _vp, _vp, _vp]),
    ("sd_cas_synth_stream_dev", _i, [_vp, _u64, _u64, _u64, _u64, _vp, _vp]),
    ("sd_cas_synth_roots_dev", _i, [_vp, _u64, _u64, _sz, _u32, _vp, _vp]),
]


def build(verbose: bool = False) -> str:
    """Compile the HIP library in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-C", CSRC, "-j", jobs] + ([] if verbose else ["-s"]), check=True)
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"build did not produce {LIB_PATH}")
    return LIB_PATH


_LIB = None


def lib() -> ctypes.CDLL:
    """Load libsd_hip_cas.so; raises if it has not been built (no silent fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: the HIP extension is the only implementation. "
                "Run spacedrive_amd._native.build() (or __graft_entry__.build()).")
        # One HIP/HSA runtime per process: torch ships its own libamdhip64.so.7, and if this
        # library were loaded first its DT_NEEDED would pull /opt/rocm's copy too — two HSA
        # runtimes in one process, and whichever opens the GPU second finds none (measured:
        # ENODEV here or "No HIP GPUs" in torch).  Loading torch first makes our SONAME
        # lookup bind to the copy already mapped.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            if os.environ.get("SD_HIP_CAS_LIB") and not hasattr(L, name):
                continue  # an older build under A/B profiling may lack newer entry points
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


class CasError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code
