// Builds libsd_hip_cas.so with hipcc (gfx950) through the repo's Makefile and links it.
use std::{env, path::PathBuf, process::Command};

fn main() {
    let root = PathBuf::from(env::var("SD_HIP_CAS_ROOT").unwrap_or_else(|_| "../..".into()));
    let csrc = root.join("spacedrive_amd/csrc");
    let status = Command::new("make")
        .arg("-C")
        .arg(&csrc)
        .arg("-j8")
        .status()
        .expect("make (hipcc) failed to start");
    assert!(status.success(), "building libsd_hip_cas.so with hipcc failed");
    println!("cargo:rustc-link-search=native={}", root.join("spacedrive_amd").display());
    println!("cargo:rustc-link-lib=dylib=sd_hip_cas");
    println!("cargo:rerun-if-changed={}", csrc.display());
    println!("cargo:rerun-if-changed={}", root.join("include/sd_hip_cas.h").display());
}
