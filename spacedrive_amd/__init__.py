"""spacedrive_amd — MI355X (gfx950) content-identification engine for Spacedrive's file
identifier: batched generate_cas_id, Object grouping and full-content checksums as
hand-written HIP kernels behind a C ABI (include/sd_hip_cas.h).  See DESIGN.md."""
from .cas import (  # noqa: F401
    CHUNK_SIZE,
    HEADER_OR_FOOTER_SIZE,
    MINIMUM_FILE_SIZE,
    NO_OBJECT,
    NO_STEP,
    SAMPLE_COUNT,
    SAMPLE_SIZE,
    SAMPLED_CONTENT_LEN,
    CasEngine,
    CasError,
    FileMetadata,
    StepResult,
    cas_id_to_key,
    engine,
    file_checksum,
    generate_cas_id,
    generate_cas_ids,
    get_ephemeral_thumb_key,
    get_ephemeral_thumbnail_path,
    get_indexed_thumb_key,
    get_indexed_thumbnail_path,
    get_shard_hex,
    identifier_job_step,
    key_to_cas_id,
    thumbnail_dir,
)

__all__ = [n for n in dir() if not n.startswith("_")]
