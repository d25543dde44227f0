// Links libmaxio_ec.so (make -C maxio_amd/csrc); MAXIO_EC_LIB_DIR points at
// maxio_amd/lib (or wherever the .so was installed).
fn main() {
    let dir = std::env::var("MAXIO_EC_LIB_DIR").unwrap_or_else(|_| "../../maxio_amd/lib".to_string());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=maxio_ec");
    println!("cargo:rerun-if-env-changed=MAXIO_EC_LIB_DIR");
}
