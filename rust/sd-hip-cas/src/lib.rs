//! Safe wrapper over libsd_hip_cas: the batched drop-in for `generate_cas_id`
//! (core/src/object/cas.rs:23-62), the Object-link decisions of the file identifier job
//! (core/src/object/file_identifier/file_identifier_job.rs:180-236, mod.rs:98-350) and
//! `file_checksum` (core/src/object/validation/hash.rs:11-25).  See INTEGRATION.md.
//!
//! The `extern "C"` block declares every entry point of include/sd_hip_cas.h;
//! tests/test_rust_binding.py checks it against the header (names, argument and return
//! types) on every CPU test run, since cargo is not available where this repo is built.
#![allow(non_camel_case_types)]
use std::{
    ffi::{c_char, c_int, c_void, CStr, CString},
    io,
    os::unix::ffi::OsStrExt,
    path::{Path, PathBuf},
    ptr,
};

#[repr(C)]
pub struct sd_cas_ctx {
    _p: [u8; 0],
}

#[repr(C)]
pub struct sd_cas_multi {
    _p: [u8; 0],
}

pub const SD_CAS_ROW_HASHED: u8 = 0;
pub const SD_CAS_ROW_NO_CAS: u8 = 1;
pub const SD_CAS_ROW_ERROR: u8 = 2;
pub const SD_CAS_LINK_CREATED: u8 = 0;
pub const SD_CAS_LINK_LINKED: u8 = 1;
pub const SD_CAS_LINK_DROPPED: u8 = 2;
pub const SD_CAS_LINK_NOT_REACHED: u8 = 3;
pub const SD_CAS_LINK_EXISTING: u8 = 4;
pub const SD_CAS_NO_OBJECT: u32 = 0xFFFF_FFFF;
pub const SD_CAS_NO_STEP: u32 = 0xFFFF_FFFF;
pub const SD_CAS_CHUNK_SIZE: u32 = 100;
/// status of a row whose fs::metadata length is 0: no cas_id (file_identifier/mod.rs:78-86)
pub const SD_CAS_STATUS_NO_CAS: i32 = 1;

extern "C" {
    pub fn sd_cas_abi_version() -> c_int;
    pub fn sd_cas_ctx_create(device: c_int, out: *mut *mut sd_cas_ctx) -> c_int;
    pub fn sd_cas_ctx_destroy(ctx: *mut sd_cas_ctx);
    pub fn sd_cas_last_error(ctx: *const sd_cas_ctx) -> *const c_char;
    pub fn sd_cas_ctx_stream(ctx: *mut sd_cas_ctx) -> *mut c_void;
    pub fn sd_cas_synchronize(ctx: *mut sd_cas_ctx) -> c_int;
    pub fn sd_cas_batch_quantum(ctx: *const sd_cas_ctx) -> usize;
    pub fn sd_cas_set_latency_threshold(ctx: *mut sd_cas_ctx, sampled_files: usize, packed_files: usize);
    pub fn sd_cas_set_chunkpar_split(ctx: *mut sd_cas_ctx, sampled_files: usize, packed_files: usize);
    pub fn sd_cas_set_group_method(ctx: *mut sd_cas_ctx, method: c_int, bucket_target: u64) -> c_int;
    pub fn sd_cas_alloc_pinned(ctx: *mut sd_cas_ctx, bytes: usize, out: *mut *mut c_void) -> c_int;
    pub fn sd_cas_free_pinned(ctx: *mut sd_cas_ctx, p: *mut c_void) -> c_int;
    pub fn sd_cas_generate_cas_ids(ctx: *mut sd_cas_ctx, bufs: *const *const u8, buf_lens: *const u64,
                                   sizes: *const u64, n: usize, out_keys: *mut u64) -> c_int;
    pub fn sd_cas_generate_cas_ids_from_paths(ctx: *mut sd_cas_ctx, paths: *const *const c_char,
                                              sizes: *const u64, n: usize, out_keys: *mut u64,
                                              status: *mut i32) -> c_int;
    pub fn sd_cas_file_metadata_from_paths(ctx: *mut sd_cas_ctx, paths: *const *const c_char, n: usize,
                                           out_keys: *mut u64, status: *mut i32,
                                           out_sizes: *mut u64) -> c_int;
    pub fn sd_cas_hash_sampled_host(ctx: *mut sd_cas_ctx, h_content: *const c_void, stride: u64,
                                    h_sizes: *const u64, n: usize, h_keys: *mut u64,
                                    batch_files: usize) -> c_int;
    pub fn sd_cas_hash_sampled_host_ring(ctx: *mut sd_cas_ctx, h_ring: *const c_void, stride: u64,
                                         ring_files: usize, h_sizes: *const u64, n: usize,
                                         h_keys: *mut u64, batch_files: usize) -> c_int;
    pub fn sd_cas_key_to_hex(key: u64, out: *mut c_char);
    pub fn sd_cas_shard_hex(key: u64, out: *mut c_char);
    pub fn sd_cas_thumbnail_path(data_dir: *const c_char, library_id: *const c_char, key: u64,
                                 out: *mut c_char, cap: usize) -> i64;
    pub fn sd_cas_thumb_key(library_id: *const c_char, key: u64, out: *mut c_char, cap: usize) -> i64;
    pub fn sd_cas_keys_to_hex_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, n: usize, d_out: *mut c_char,
                                  stream: *mut c_void) -> c_int;
    pub fn sd_cas_thumbnail_paths_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, n: usize,
                                      prefix: *const c_char, stride: u32, d_out: *mut c_char,
                                      stream: *mut c_void) -> c_int;
    pub fn sd_cas_hash_sampled_dev(ctx: *mut sd_cas_ctx, d_content: *const c_void, stride: u64,
                                   d_sizes: *const u64, n: usize, d_keys: *mut u64,
                                   stream: *mut c_void) -> c_int;
    pub fn sd_cas_hash_packed_dev(ctx: *mut sd_cas_ctx, d_arena: *const c_void, d_offs: *const u64,
                                  d_lens: *const u32, d_sizes: *const u64, n: usize, d_keys: *mut u64,
                                  stream: *mut c_void) -> c_int;
    pub fn sd_cas_group_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, n: usize, d_rep: *mut u32,
                            out_objects: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_hash_group_sampled_dev(ctx: *mut sd_cas_ctx, d_content: *const c_void, stride: u64,
                                         d_sizes: *const u64, n: usize, d_keys: *mut u64,
                                         d_rep: *mut u32, d_overflow: *mut u32,
                                         out_objects: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_hash_regions_sampled_dev(ctx: *mut sd_cas_ctx, d_content: *const c_void, stride: u64,
                                           d_sizes: *const u64, n: usize, d_keys: *mut u64,
                                           d_rep: *mut u32, d_overflow: *mut u32,
                                           stream: *mut c_void) -> c_int;
    pub fn sd_cas_group_regions_dev(ctx: *mut sd_cas_ctx, n: usize, d_rep: *mut u32,
                                    out_objects: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_group_min_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, d_vals: *const u32, n: usize,
                                d_out: *mut u32, out_objects: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_partition_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, n: usize, parts: u32,
                                d_keys_out: *mut u64, d_pos_out: *mut u32, d_counts: *mut u64,
                                stream: *mut c_void) -> c_int;
    pub fn sd_cas_exchange_pack_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, d_pos: *const u32,
                                    n: usize, file0: u64, d_rows: *mut u32, stream: *mut c_void) -> c_int;
    pub fn sd_cas_exchange_split_dev(ctx: *mut sd_cas_ctx, d_rows: *const u32, m: usize,
                                     d_keys: *mut u64, d_vals: *mut u32, stream: *mut c_void) -> c_int;
    pub fn sd_cas_exchange_unpack_dev(ctx: *mut sd_cas_ctx, d_back: *const u32, d_pos: *const u32,
                                      n: usize, d_rep: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_exchange_pack_fixed_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, d_pos: *const u32,
                                          d_counts: *const u64, G: u32, cap: u64, spill: u64,
                                          file0: u64, d_rows: *mut u32, d_spill_rows: *mut u32,
                                          d_overflow: *mut u32, stream: *mut c_void) -> c_int;
    pub fn sd_cas_exchange_split_fixed_dev(ctx: *mut sd_cas_ctx, d_rows: *const u32, m: usize,
                                           sentinel: u64, d_keys: *mut u64, d_vals: *mut u32,
                                           d_sentinel_rows: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_exchange_unpack_fixed_dev(ctx: *mut sd_cas_ctx, d_back: *const u32,
                                            d_spill_back: *const u32, d_pos: *const u32,
                                            d_counts: *const u64, G: u32, cap: u64, spill: u64,
                                            d_rep: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_copy_objects_dev(ctx: *mut sd_cas_ctx, d_dst: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_group_sorted_dev(ctx: *mut sd_cas_ctx, d_sorted_keys: *const u64,
                                   d_sorted_vals: *const u32, n: usize, d_rep: *mut u32,
                                   out_objects: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_group_chunked_dev(ctx: *mut sd_cas_ctx, d_rep: *const u32, n: usize, chunk: u32,
                                    d_rep_chunked: *mut u32, out_created: *mut u64,
                                    out_linked: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_identifier_max_steps(n: usize, chunk: u32) -> usize;
    pub fn sd_cas_identifier_links_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, d_state: *const u8,
                                       n: usize, chunk: u32, d_step: *mut u32, d_object: *mut u32,
                                       d_action: *mut u8, h_step_counts: *mut u64, max_steps: usize,
                                       out_steps: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_identifier_links(ctx: *mut sd_cas_ctx, h_keys: *const u64, h_state: *const u8,
                                   n: usize, chunk: u32, h_step: *mut u32, h_object: *mut u32,
                                   h_action: *mut u8, h_step_counts: *mut u64, max_steps: usize,
                                   out_steps: *mut u64) -> c_int;
    pub fn sd_cas_identifier_links_seeded_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, d_state: *const u8,
                                              n: usize, chunk: u32, d_seed_keys: *const u64,
                                              d_seed_objects: *const u32, n_seed: usize,
                                              d_step: *mut u32, d_object: *mut u32, d_action: *mut u8,
                                              h_step_counts: *mut u64, max_steps: usize,
                                              out_steps: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_identifier_links_seeded(ctx: *mut sd_cas_ctx, h_keys: *const u64, h_state: *const u8,
                                          n: usize, chunk: u32, h_seed_keys: *const u64,
                                          h_seed_objects: *const u32, n_seed: usize, h_step: *mut u32,
                                          h_object: *mut u32, h_action: *mut u8,
                                          h_step_counts: *mut u64, max_steps: usize,
                                          out_steps: *mut u64) -> c_int;
    pub fn sd_cas_identifier_links_ex_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, d_state: *const u8,
                                          n: usize, chunk: u32, d_seed_keys: *const u64,
                                          d_seed_objects: *const u32, n_seed: usize,
                                          d_pre_objects: *const u32, d_step: *mut u32,
                                          d_object: *mut u32, d_action: *mut u8,
                                          h_step_counts: *mut u64, max_steps: usize,
                                          out_steps: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_identifier_links_ex(ctx: *mut sd_cas_ctx, h_keys: *const u64, h_state: *const u8,
                                      n: usize, chunk: u32, h_seed_keys: *const u64,
                                      h_seed_objects: *const u32, n_seed: usize,
                                      h_pre_objects: *const u32, h_step: *mut u32,
                                      h_object: *mut u32, h_action: *mut u8,
                                      h_step_counts: *mut u64, max_steps: usize,
                                      out_steps: *mut u64) -> c_int;
    pub fn sd_cas_sort_pairs_dev(ctx: *mut sd_cas_ctx, d_keys_in: *const u64, d_vals_in: *const u32,
                                 n: usize, d_keys_out: *mut u64, d_vals_out: *mut u32, begin_bit: c_int,
                                 end_bit: c_int, stream: *mut c_void) -> c_int;
    pub fn sd_cas_checksum_dev(ctx: *mut sd_cas_ctx, d_data: *const c_void, len: u64, out: *mut u8,
                               stream: *mut c_void) -> c_int;
    pub fn sd_cas_file_checksum(ctx: *mut sd_cas_ctx, path: *const c_char, out_hex: *mut c_char,
                                err_no: *mut c_int) -> c_int;
    pub fn sd_cas_checksums_dev(ctx: *mut sd_cas_ctx, d_arena: *const c_void, arena_bytes: u64,
                                d_offs: *const u64, d_lens: *const u64, n: usize, d_out: *mut u8,
                                stream: *mut c_void) -> c_int;
    pub fn sd_cas_file_checksums(ctx: *mut sd_cas_ctx, paths: *const *const c_char, n: usize,
                                 out_hex: *mut c_char, status: *mut i32) -> c_int;
    pub fn sd_cas_multi_create(devices: *const c_int, ndev: c_int, out: *mut *mut sd_cas_multi) -> c_int;
    pub fn sd_cas_multi_destroy(m: *mut sd_cas_multi);
    pub fn sd_cas_multi_count(m: *const sd_cas_multi) -> c_int;
    pub fn sd_cas_multi_ctx(m: *mut sd_cas_multi, i: c_int) -> *mut sd_cas_ctx;
    pub fn sd_cas_multi_last_error(m: *const sd_cas_multi) -> *const c_char;
    pub fn sd_cas_multi_group(m: *mut sd_cas_multi, d_keys: *const *const u64, n: *const usize,
                              file0: *const u64, d_rep: *const *mut u64, out_objects: *mut u64) -> c_int;
    pub fn sd_cas_multi_hash_group_sampled_host(m: *mut sd_cas_multi, h_content: *const c_void,
                                                stride: u64, h_sizes: *const u64, n: usize,
                                                h_keys: *mut u64, h_rep: *mut u64,
                                                out_objects: *mut u64) -> c_int;
    pub fn sd_cas_synth_sampled_dev(ctx: *mut sd_cas_ctx, seed: u64, file0: u64, n: usize,
                                    dup_permille: u32, d_content: *mut c_void, stride: u64,
                                    d_sizes: *mut u64, stream: *mut c_void) -> c_int;
    pub fn sd_cas_synth_small_dev(ctx: *mut sd_cas_ctx, seed: u64, file0: u64, n: usize,
                                  dup_permille: u32, d_sizes: *mut u64, d_lens: *mut u32,
                                  d_offs: *mut u64, d_arena: *mut c_void, out_arena_bytes: *mut u64,
                                  stream: *mut c_void) -> c_int;
    pub fn sd_cas_synth_small_content_dev(ctx: *mut sd_cas_ctx, seed: u64, file0: u64, n: usize,
                                          dup_permille: u32, d_offs: *const u64, d_lens: *const u32,
                                          d_arena: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn sd_cas_synth_stream_dev(ctx: *mut sd_cas_ctx, seed: u64, file: u64, byte_off: u64,
                                   len: u64, d_out: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn sd_cas_synth_roots_dev(ctx: *mut sd_cas_ctx, seed: u64, file0: u64, n: usize,
                                  dup_permille: u32, d_roots: *mut u64, stream: *mut c_void) -> c_int;
}

/// A cas_id: the big-endian u64 of BLAKE3(le64(size) || content)[0..8].
/// `to_string()` is the 16-char lowercase hex `String` of cas.rs:61.
#[derive(Clone, Copy, Debug, PartialEq, Eq, Hash, PartialOrd, Ord)]
pub struct CasId(pub u64);

impl std::fmt::Display for CasId {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "{:016x}", self.0)
    }
}

impl CasId {
    /// get_shard_hex (thumbnail/shard.rs:10-13) through sd_cas_shard_hex.
    pub fn shard_hex(&self) -> String {
        let mut out = [0 as c_char; 4];
        unsafe { sd_cas_shard_hex(self.0, out.as_mut_ptr()) };
        unsafe { CStr::from_ptr(out.as_ptr()) }.to_string_lossy().into_owned()
    }

    /// get_thumbnail_path (thumbnail/mod.rs:67-82): `library` None = ThumbnailKind::Ephemeral.
    pub fn thumbnail_path(&self, data_dir: &Path, library: Option<&str>) -> PathBuf {
        let dd = CString::new(data_dir.as_os_str().as_encoded_bytes()).expect("NUL in path");
        let lib = library.map(|l| CString::new(l).expect("NUL in library id"));
        let lp = lib.as_ref().map_or(ptr::null(), |l| l.as_ptr());
        let need = unsafe { sd_cas_thumbnail_path(dd.as_ptr(), lp, self.0, ptr::null_mut(), 0) };
        let mut buf = vec![0 as c_char; need as usize + 1];
        unsafe { sd_cas_thumbnail_path(dd.as_ptr(), lp, self.0, buf.as_mut_ptr(), buf.len()) };
        let s = unsafe { CStr::from_ptr(buf.as_ptr()) };
        PathBuf::from(std::ffi::OsStr::from_bytes(s.to_bytes()))  // Unix paths are bytes
    }
}

/// What happens to one orphan row in the job (sd_cas_identifier_links).
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub enum RowState {
    /// cas_id computed
    Hashed(CasId),
    /// fs::metadata length 0: no cas_id, its own Object (mod.rs:78-86)
    NoCas,
    /// FileMetadata::new failed: logged and dropped from the step (mod.rs:125-141)
    Error,
}

/// One orphan row with the Object its file_path may already hold: the orphan query is
/// `object_id IS NULL OR cas_id IS NULL` (file_identifier_job.rs:258-261), so a file the
/// watcher gave an Object while it was empty and that was written since (object_id set,
/// cas_id NULL; watcher/utils.rs:236-293, 473-490) is a row too.  `object` = that Object's
/// id (< 2^31, the DB's row order), `None` for the usual row.
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub struct OrphanRow {
    pub state: RowState,
    pub object: Option<u32>,
}

/// One job step's DB batches (mod.rs:157-347): `creates` feed `create_many` + the link
/// updates of the new Objects, `links` connect rows to the Object created for `.1`,
/// `links_existing` connect rows to an Object that existed before the job (`.1` = its id as
/// given in `ExistingObject`, mod.rs:202-238).
#[derive(Clone, Debug, Default, PartialEq, Eq)]
pub struct StepBatch {
    pub creates: Vec<usize>,
    pub links: Vec<(usize, usize)>,
    pub links_existing: Vec<(usize, u32)>,
    pub total_created: u64,
    pub total_linked: u64,
}

/// An Object the library holds before the job, as the step's `find_many` would return it
/// (mod.rs:180-198): one pair per (Object, cas_id of one of its file_paths).  `id` < 2^31,
/// ascending in the DB's row order (`find()` picks the smallest, mod.rs:214-224).
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub struct ExistingObject {
    pub cas_id: CasId,
    pub id: u32,
}

/// One context per (job thread, device).  Not Sync; Send is fine.
pub struct HipCas {
    ctx: *mut sd_cas_ctx,
}
unsafe impl Send for HipCas {}

impl HipCas {
    pub fn new(device: i32) -> io::Result<Self> {
        let mut ctx = ptr::null_mut();
        let rc = unsafe { sd_cas_ctx_create(device, &mut ctx) };
        if rc != 0 {
            return Err(io::Error::other(format!("sd_cas_ctx_create({device}) = {rc}")));
        }
        Ok(Self { ctx })
    }

    fn err(&self, rc: c_int) -> io::Error {
        let msg = unsafe { CStr::from_ptr(sd_cas_last_error(self.ctx)) };
        io::Error::other(format!("sd-hip-cas ({rc}): {}", msg.to_string_lossy()))
    }

    /// North-star drop-in: `generate_cas_ids(&[(buf, size)]) -> Vec<CasId>`.
    /// `buf` = whole file (size <= 100 KiB) or the 57,344 gathered sample bytes.
    pub fn generate_cas_ids(&mut self, items: &[(&[u8], u64)]) -> io::Result<Vec<CasId>> {
        let bufs: Vec<*const u8> = items.iter().map(|(b, _)| b.as_ptr()).collect();
        let lens: Vec<u64> = items.iter().map(|(b, _)| b.len() as u64).collect();
        let sizes: Vec<u64> = items.iter().map(|(_, s)| *s).collect();
        let mut keys = vec![0u64; items.len()];
        let rc = unsafe {
            sd_cas_generate_cas_ids(self.ctx, bufs.as_ptr(), lens.as_ptr(), sizes.as_ptr(),
                                    items.len(), keys.as_mut_ptr())
        };
        if rc != 0 {
            return Err(self.err(rc));
        }
        Ok(keys.into_iter().map(CasId).collect())
    }

    /// The cas part of `FileMetadata::new` (file_identifier/mod.rs:55-95) over a batch:
    /// gather (cas.rs:27-58 offsets) + hash.  `size` = the `fs::metadata().len()` just read.
    /// Per file: `Ok(Some(cas_id))`, `Ok(None)` for length 0 (no cas_id, mod.rs:78-86), or the
    /// io error (a directory is `EISDIR`; the reference asserts, mod.rs:67-70).
    pub fn generate_cas_ids_from_paths(&mut self, files: &[(&Path, u64)])
        -> io::Result<Vec<Result<Option<CasId>, io::Error>>> {
        let paths: Vec<&Path> = files.iter().map(|(p, _)| *p).collect();
        let sizes: Vec<u64> = files.iter().map(|(_, s)| *s).collect();
        self.cas_ids_from_paths(&paths, Some(&sizes))
    }

    /// Same with the metadata taken by the library (stat, following symlinks like
    /// `fs::metadata`, mod.rs:63): `FileMetadata::new`'s cas_id for each path.
    pub fn file_metadata_cas_ids(&mut self, paths: &[&Path])
        -> io::Result<Vec<Result<Option<CasId>, io::Error>>> {
        self.cas_ids_from_paths(paths, None)
    }

    fn cas_ids_from_paths(&mut self, paths: &[&Path], sizes: Option<&[u64]>)
        -> io::Result<Vec<Result<Option<CasId>, io::Error>>> {
        let cpaths: Vec<CString> = paths
            .iter()
            .map(|p| CString::new(p.as_os_str().as_encoded_bytes()).expect("NUL in path"))
            .collect();
        let ptrs: Vec<*const c_char> = cpaths.iter().map(|c| c.as_ptr()).collect();
        let mut keys = vec![0u64; paths.len()];
        let mut status = vec![0i32; paths.len()];
        let rc = unsafe {
            sd_cas_generate_cas_ids_from_paths(self.ctx, ptrs.as_ptr(),
                                               sizes.map_or(ptr::null(), |s| s.as_ptr()), paths.len(),
                                               keys.as_mut_ptr(), status.as_mut_ptr())
        };
        if rc != 0 {
            return Err(self.err(rc));
        }
        Ok(keys
            .into_iter()
            .zip(status)
            .map(|(k, s)| match s {
                0 => Ok(Some(CasId(k))),
                SD_CAS_STATUS_NO_CAS => Ok(None),
                e => Err(io::Error::from_raw_os_error(-e)),
            })
            .collect())
    }

    /// `FileMetadata::new` over a batch with the metadata taken by the library: per path the
    /// cas_id result and the `fs::metadata().len()` it was decided from (one stat per path).
    pub fn file_metadata(&mut self, paths: &[&Path])
        -> io::Result<Vec<(Result<Option<CasId>, io::Error>, u64)>> {
        let cpaths: Vec<CString> = paths
            .iter()
            .map(|p| CString::new(p.as_os_str().as_encoded_bytes()).expect("NUL in path"))
            .collect();
        let ptrs: Vec<*const c_char> = cpaths.iter().map(|c| c.as_ptr()).collect();
        let n = paths.len();
        let (mut keys, mut status, mut sizes) = (vec![0u64; n], vec![0i32; n], vec![0u64; n]);
        let rc = unsafe {
            sd_cas_file_metadata_from_paths(self.ctx, ptrs.as_ptr(), n, keys.as_mut_ptr(),
                                            status.as_mut_ptr(), sizes.as_mut_ptr())
        };
        if rc != 0 {
            return Err(self.err(rc));
        }
        Ok((0..n)
            .map(|i| {
                let r = match status[i] {
                    0 => Ok(Some(CasId(keys[i]))),
                    SD_CAS_STATUS_NO_CAS => Ok(None),
                    e => Err(io::Error::from_raw_os_error(-e)),
                };
                (r, sizes[i])
            })
            .collect())
    }

    /// The Object decisions of a whole file-identifier job over `rows` (orphan file_paths in
    /// ascending id order, fresh library), `chunk` rows per step with the reference's cursor:
    /// the batches each step hands to the DB (file_identifier_job.rs:180-236, mod.rs:157-347).
    pub fn identifier_links(&mut self, rows: &[RowState], chunk: u32) -> io::Result<Vec<StepBatch>> {
        self.identifier_links_existing(rows, chunk, &[])
    }

    /// The same job on a library that already holds Objects (`existing`: every Object
    /// connected to a file_path with some cas_id, from the DB): a row whose cas_id one of them
    /// carries links to the smallest such id in `links_existing` and its key never creates
    /// (mod.rs:180-253; the query has no location filter).
    pub fn identifier_links_existing(&mut self, rows: &[RowState], chunk: u32,
                                     existing: &[ExistingObject]) -> io::Result<Vec<StepBatch>> {
        let orphans: Vec<OrphanRow> = rows.iter().map(|&state| OrphanRow { state, object: None }).collect();
        self.identifier_links_orphans(&orphans, chunk, existing)
    }

    /// The general job: rows may already own an Object (`OrphanRow::object`).  The step that
    /// processes such a Hashed row writes its cas_id first, so its find_many (mod.rs:157-198)
    /// also returns that Object: every row of the step with the cas_id links to the smallest
    /// Object id carrying it (`links_existing`, the row itself included) and the cas_id never
    /// creates (mod.rs:202-253) — sd_cas_identifier_links_ex.
    pub fn identifier_links_orphans(&mut self, rows: &[OrphanRow], chunk: u32,
                                    existing: &[ExistingObject]) -> io::Result<Vec<StepBatch>> {
        let n = rows.len();
        let keys: Vec<u64> = rows.iter().map(|r| if let RowState::Hashed(k) = r.state { k.0 } else { 0 }).collect();
        let state: Vec<u8> = rows
            .iter()
            .map(|r| match r.state {
                RowState::Hashed(_) => SD_CAS_ROW_HASHED,
                RowState::NoCas => SD_CAS_ROW_NO_CAS,
                RowState::Error => SD_CAS_ROW_ERROR,
            })
            .collect();
        let pre: Option<Vec<u32>> = rows
            .iter()
            .any(|r| r.object.is_some())
            .then(|| rows.iter().map(|r| r.object.unwrap_or(SD_CAS_NO_OBJECT)).collect());
        let max_steps = unsafe { sd_cas_identifier_max_steps(n, chunk) };
        let (mut step, mut object, mut action) = (vec![0u32; n], vec![0u32; n], vec![0u8; n]);
        let mut counts = vec![0u64; 2 * max_steps.max(1)];
        let mut steps = 0u64;
        let seed_keys: Vec<u64> = existing.iter().map(|e| e.cas_id.0).collect();
        let seed_ids: Vec<u32> = existing.iter().map(|e| e.id).collect();
        let rc = unsafe {
            sd_cas_identifier_links_ex(self.ctx, keys.as_ptr(), state.as_ptr(), n, chunk,
                                       seed_keys.as_ptr(), seed_ids.as_ptr(), existing.len(),
                                       pre.as_ref().map_or(ptr::null(), |p| p.as_ptr()),
                                       step.as_mut_ptr(), object.as_mut_ptr(), action.as_mut_ptr(),
                                       counts.as_mut_ptr(), max_steps, &mut steps)
        };
        if rc != 0 {
            return Err(self.err(rc));
        }
        let mut out: Vec<StepBatch> = (0..steps as usize)
            .map(|k| StepBatch { total_created: counts[2 * k], total_linked: counts[2 * k + 1], ..Default::default() })
            .collect();
        for i in 0..n {
            match action[i] {
                SD_CAS_LINK_CREATED => out[step[i] as usize].creates.push(i),
                SD_CAS_LINK_LINKED => out[step[i] as usize].links.push((i, object[i] as usize)),
                SD_CAS_LINK_EXISTING => out[step[i] as usize].links_existing.push((i, object[i])),
                _ => {}
            }
        }
        // A NoCas row that ends a chunk stays orphan (cas_id NULL), so the next step's
        // `id >= cursor` query returns it again and it gets an Object in BOTH steps
        // (mod.rs:277-283, 401-405); `step` holds its last step only.  The row missing from
        // step k's creates is the first row of step k+1 (the cursor row): the smallest row
        // whose last step is after k — processed rows' steps are non-decreasing in row order.
        let mut first = 0usize;
        for k in 0..out.len() {
            if out[k].total_created as usize > out[k].creates.len() {
                while first < n && (step[first] == SD_CAS_NO_STEP || step[first] as usize <= k) {
                    first += 1;
                }
                if first < n {
                    out[k].creates.push(first);
                }
            }
        }
        Ok(out)
    }

    /// `file_checksum(path)` (validation/hash.rs:11).
    pub fn file_checksum(&mut self, path: &Path) -> io::Result<String> {
        let c = CString::new(path.as_os_str().as_encoded_bytes()).expect("NUL in path");
        let mut out = [0 as c_char; 65];
        let mut e: c_int = 0;
        let rc = unsafe { sd_cas_file_checksum(self.ctx, c.as_ptr(), out.as_mut_ptr(), &mut e) };
        if rc == -3 && e != 0 {
            return Err(io::Error::from_raw_os_error(e));
        }
        if rc != 0 {
            return Err(self.err(rc));
        }
        Ok(unsafe { CStr::from_ptr(out.as_ptr()) }.to_string_lossy().into_owned())
    }

    /// The validator job's checksums over many files in one call (`sd_cas_file_checksums`):
    /// one `io::Result` per path, as `file_checksum` would return it.
    pub fn file_checksums(&mut self, paths: &[&Path]) -> io::Result<Vec<io::Result<String>>> {
        let cs: Vec<CString> = paths
            .iter()
            .map(|p| CString::new(p.as_os_str().as_encoded_bytes()).expect("NUL in path"))
            .collect();
        let ptrs: Vec<*const c_char> = cs.iter().map(|c| c.as_ptr()).collect();
        let n = paths.len();
        let mut out = vec![0 as c_char; 65 * n.max(1)];
        let mut status = vec![0i32; n];
        let rc = unsafe {
            sd_cas_file_checksums(self.ctx, ptrs.as_ptr(), n, out.as_mut_ptr(), status.as_mut_ptr())
        };
        if rc != 0 {
            return Err(self.err(rc));
        }
        Ok((0..n)
            .map(|i| {
                if status[i] != 0 {
                    Err(io::Error::from_raw_os_error(-status[i]))
                } else {
                    Ok(unsafe { CStr::from_ptr(out.as_ptr().add(65 * i)) }.to_string_lossy().into_owned())
                }
            })
            .collect())
    }

    /// Canonical Object grouping of device-resident keys (see `sd_cas_group_dev`); returns
    /// the number of Objects.  `d_keys`/`d_rep` are device pointers owned by the caller.
    ///
    /// # Safety
    /// `d_keys` must point to `n` u64 and `d_rep` to `n` u32 in device memory of this
    /// context's GPU.
    pub unsafe fn group_dev(&mut self, d_keys: *const u64, n: usize, d_rep: *mut u32) -> io::Result<u64> {
        let mut objects = 0u64;
        let rc = sd_cas_group_dev(self.ctx, d_keys, n, d_rep, &mut objects, ptr::null_mut());
        if rc != 0 {
            return Err(self.err(rc));
        }
        Ok(objects)
    }

    /// The 100-row chunk replay of a canonical grouping (`sd_cas_group_chunked_dev`):
    /// returns the summed (total_created, total_linked) of mod.rs:349.
    ///
    /// # Safety
    /// `d_rep` / `d_rep_chunked` must point to `n` u32 in device memory of this context's GPU.
    pub unsafe fn group_chunked_dev(&mut self, d_rep: *const u32, n: usize, chunk: u32,
                                    d_rep_chunked: *mut u32) -> io::Result<(u64, u64)> {
        let (mut created, mut linked) = (0u64, 0u64);
        let rc = sd_cas_group_chunked_dev(self.ctx, d_rep, n, chunk, d_rep_chunked, &mut created,
                                          &mut linked, ptr::null_mut());
        if rc != 0 {
            return Err(self.err(rc));
        }
        Ok((created, linked))
    }
}

impl Drop for HipCas {
    fn drop(&mut self) {
        unsafe { sd_cas_ctx_destroy(self.ctx) }
    }
}
