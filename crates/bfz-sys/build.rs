// Links libbfz.so (built by `make -C zkvm-brainfuck_amd`, hipcc --offload-arch=gfx950).
// BFZ_LIB_DIR points at the directory holding libbfz.so; the rpath lets test binaries find it.
fn main() {
    let dir = std::env::var("BFZ_LIB_DIR").unwrap_or_else(|_| {
        let root = std::path::Path::new(env!("CARGO_MANIFEST_DIR")).join("../../zkvm-brainfuck_amd");
        root.to_string_lossy().into_owned()
    });
    println!("cargo:rerun-if-env-changed=BFZ_LIB_DIR");
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=bfz");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
}
