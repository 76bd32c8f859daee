// Link libsdrgpu.so from this repository's build (make -C unnamed-rust-sdr_amd); override
// with SDRGPU_LIB_DIR.  libsdrgpu.so itself pulls in the ROCm runtime and RCCL.
fn main() {
    let dir = std::env::var("SDRGPU_LIB_DIR").unwrap_or_else(|_| {
        let here = std::env::var("CARGO_MANIFEST_DIR").unwrap();
        format!("{}/../../unnamed-rust-sdr_amd", here)
    });
    println!("cargo:rustc-link-search=native={}", dir);
    println!("cargo:rustc-link-lib=dylib=sdrgpu");
    println!("cargo:rerun-if-env-changed=SDRGPU_LIB_DIR");
}
