// Links the hipcc-built static archive (diamond-types_amd/Makefile `static` target:
// lib/libdtgpu.a, one gfx950 code object per translation unit, no device-link step) and the
// HIP runtime it calls.  Same shape as crates/dt-swift/build.rs in the reference.
use std::env;
use std::path::PathBuf;
use std::process::Command;

fn main() {
    let root = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../../diamond-types_amd");
    let rocm = env::var("ROCM_PATH").unwrap_or_else(|_| "/opt/rocm".to_string());
    // build the archive with the in-tree Makefile (hipcc --offload-arch=gfx950)
    let st = Command::new("make").arg("-C").arg(&root).arg("static").status().expect("make");
    assert!(st.success(), "make static failed");
    println!("cargo:rustc-link-search=native={}", root.join("lib").display());
    println!("cargo:rustc-link-lib=static=dtgpu");
    println!("cargo:rustc-link-search=native={}/lib", rocm);
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    println!("cargo:rustc-link-lib=dylib=stdc++");
    println!("cargo:rerun-if-changed={}", root.join("csrc").display());
    println!("cargo:rerun-if-changed=../../include/dtgpu.h");
}
