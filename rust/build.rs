// Links libspai.so (make -C self-play-ai_amd) and the ROCm runtime it needs.
// SPAI_LIB_DIR points at the directory holding libspai.so.
fn main() {
    let dir = std::env::var("SPAI_LIB_DIR").unwrap_or_else(|_| "../self-play-ai_amd".to_string());
    println!("cargo:rustc-link-search=native={}", dir);
    println!("cargo:rustc-link-lib=dylib=spai");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir);
    println!("cargo:rustc-link-arg=-Wl,-rpath,/opt/rocm/lib");
    println!("cargo:rerun-if-env-changed=SPAI_LIB_DIR");
}
