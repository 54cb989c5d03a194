//! Builds libpbft_verify.so for gfx950 with exactly the compiler lines of
//! `__graft_entry__.build()` and links it.
//!
//! NOT COMPILED HERE (no Rust toolchain in the image).  Environment:
//!   PBFT_SRC   path of this repository's checkout (default: `..` of the crate)
//!   HIPCC      hipcc binary (default /opt/rocm/bin/hipcc); ROCM_PATH for libamdhip64
use std::env;
use std::path::PathBuf;
use std::process::Command;

fn run(cmd: &mut Command) {
    let status = cmd.status().unwrap_or_else(|e| panic!("failed to spawn {:?}: {}", cmd, e));
    assert!(status.success(), "command failed: {:?}", cmd);
}

fn main() {
    let crate_dir = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let src = env::var("PBFT_SRC").map(PathBuf::from).unwrap_or_else(|_| crate_dir.join(".."));
    let out = PathBuf::from(env::var("OUT_DIR").unwrap());
    let hipcc = env::var("HIPCC").unwrap_or_else(|_| "/opt/rocm/bin/hipcc".into());
    let rocm = env::var("ROCM_PATH").unwrap_or_else(|_| "/opt/rocm".into());
    let host = src.join("pbft_amd/csrc/host");

    // host-side state machine and wire codec (plain C++17)
    let mut objs = Vec::new();
    for name in ["replica", "wire"].iter() {
        let obj = out.join(format!("{}.o", name));
        run(Command::new("g++")
            .args(&["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-c", "-o"])
            .arg(&obj)
            .arg(host.join(format!("{}.cpp", name))));
        objs.push(obj);
    }
    // HIP kernels + C ABI, gfx950 code objects only (no dual paths, no other targets): one object per
    // source (the four key plans' verify kernels are separate units), then one -shared link
    let hip_sources = ["pbft_verify.hip", "tables.hip", "finish.hip", "sign.hip", "comb_pa13.hip", "comb_pa14.hip", "comb_pa16.hip", "comb_pa32.hip"];
    for name in hip_sources.iter() {
        let obj = out.join(name.replace(".hip", ".o"));
        run(Command::new(&hipcc)
            .args(&["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-c", "-o"])
            .arg(&obj)
            .arg(src.join("pbft_amd/csrc").join(name)));
        objs.insert(0, obj);
    }
    let lib = out.join("libpbft_verify.so");
    run(Command::new(&hipcc)
        .args(&["--offload-arch=gfx950", "-fPIC", "-shared", "-o"])
        .arg(&lib)
        .args(&objs));

    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=pbft_verify");
    println!("cargo:rustc-link-search=native={}/lib", rocm);
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", out.display());
    for f in ["pbft_amd/csrc/pbft_verify.hip", "pbft_amd/csrc/verify_kernels.h", "pbft_amd/csrc/host/replica.cpp", "pbft_amd/csrc/host/wire.cpp",
              "include/pbft_verify.h", "include/pbft_replica.h", "include/pbft_wire.h"].iter() {
        println!("cargo:rerun-if-changed={}", src.join(f).display());
    }
    println!("cargo:rerun-if-changed={}", src.join("pbft_amd/csrc").display());
    println!("cargo:rerun-if-env-changed=PBFT_SRC");
}
