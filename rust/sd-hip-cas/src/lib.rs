//! Safe wrapper over libsd_hip_cas: the batched drop-in for
//! `generate_cas_id` (core/src/object/cas.rs:23-62) and `file_checksum`
//! (core/src/object/validation/hash.rs:11-25).  See INTEGRATION.md.
use std::{ffi::{c_char, c_int, c_void, CStr, CString}, io, path::Path, ptr};

#[repr(C)]
pub struct sd_cas_ctx {
    _p: [u8; 0],
}

extern "C" {
    fn sd_cas_ctx_create(device: c_int, out: *mut *mut sd_cas_ctx) -> c_int;
    fn sd_cas_ctx_destroy(ctx: *mut sd_cas_ctx);
    fn sd_cas_last_error(ctx: *const sd_cas_ctx) -> *const c_char;
    fn sd_cas_generate_cas_ids(ctx: *mut sd_cas_ctx, bufs: *const *const u8, buf_lens: *const u64,
                               sizes: *const u64, n: usize, out_keys: *mut u64) -> c_int;
    fn sd_cas_generate_cas_ids_from_paths(ctx: *mut sd_cas_ctx, paths: *const *const c_char,
                                          sizes: *const u64, n: usize, out_keys: *mut u64,
                                          status: *mut i32) -> c_int;
    fn sd_cas_file_checksum(ctx: *mut sd_cas_ctx, path: *const c_char, out_hex: *mut c_char,
                            err_no: *mut c_int) -> c_int;
    fn sd_cas_group_dev(ctx: *mut sd_cas_ctx, d_keys: *const u64, n: usize, d_rep: *mut u32,
                        out_objects: *mut u64, stream: *mut c_void) -> c_int;
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

    /// Gather (cas.rs:27-58 offsets) + hash; per-file io errors like FileMetadata::new.
    pub fn generate_cas_ids_from_paths(&mut self, files: &[(&Path, u64)])
        -> io::Result<Vec<Result<CasId, io::Error>>> {
        let cpaths: Vec<CString> = files
            .iter()
            .map(|(p, _)| CString::new(p.as_os_str().as_encoded_bytes()).expect("NUL in path"))
            .collect();
        let ptrs: Vec<*const c_char> = cpaths.iter().map(|c| c.as_ptr()).collect();
        let sizes: Vec<u64> = files.iter().map(|(_, s)| *s).collect();
        let mut keys = vec![0u64; files.len()];
        let mut status = vec![0i32; files.len()];
        let rc = unsafe {
            sd_cas_generate_cas_ids_from_paths(self.ctx, ptrs.as_ptr(), sizes.as_ptr(), files.len(),
                                               keys.as_mut_ptr(), status.as_mut_ptr())
        };
        if rc != 0 {
            return Err(self.err(rc));
        }
        Ok(keys
            .into_iter()
            .zip(status)
            .map(|(k, s)| if s == 0 { Ok(CasId(k)) } else { Err(io::Error::from_raw_os_error(-s)) })
            .collect())
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
}

impl Drop for HipCas {
    fn drop(&mut self) {
        unsafe { sd_cas_ctx_destroy(self.ctx) }
    }
}
