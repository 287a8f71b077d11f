//! Builds the gfx950 engine in-tree (`make -C <repo>/grandine_amd`, hipcc
//! `--offload-arch=gfx950`) and links `libgrandine_bls.so`.  The repository root is
//! `GBLS_REPO` when set, else two levels above this crate (`rust/bls_gpu_sys`).
use std::{env, path::PathBuf, process::Command};

fn main() {
    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").expect("cargo sets CARGO_MANIFEST_DIR"));
    let repo = env::var_os("GBLS_REPO").map(PathBuf::from).unwrap_or_else(|| manifest.join("../.."));
    let engine = repo.join("grandine_amd");
    let jobs = env::var("NUM_JOBS").unwrap_or_else(|_| "8".into());
    let status = Command::new("make")
        .arg("-C")
        .arg(&engine)
        .arg(format!("-j{jobs}"))
        .status()
        .expect("make (hipcc from /opt/rocm) must be on PATH");
    assert!(status.success(), "building {} failed", engine.display());
    let lib = engine.join("lib");
    println!("cargo:rustc-link-search=native={}", lib.display());
    println!("cargo:rustc-link-lib=dylib=grandine_bls");
    // the node finds the library next to the binary or through this rpath
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", lib.display());
    println!("cargo:rerun-if-changed={}", engine.join("csrc").display());
    println!("cargo:rerun-if-changed={}", repo.join("include/grandine_bls_gpu.h").display());
    println!("cargo:rerun-if-env-changed=GBLS_REPO");
}
