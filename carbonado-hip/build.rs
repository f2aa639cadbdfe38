//! Link libcarbonado_hip.so (built in-tree by `python -c 'import
//! __graft_entry__ as g; g.build()'` into carbonado_amd/lib/).  Override the
//! directory with CARBONADO_HIP_LIB_DIR.  The library NEEDs the HIP runtime
//! (libamdhip64.so.7) and libcrypto; both resolve through the usual loader
//! paths of a ROCm install.
use std::env;
use std::path::PathBuf;

fn main() {
    let dir = match env::var("CARBONADO_HIP_LIB_DIR") {
        Ok(d) => PathBuf::from(d),
        Err(_) => PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../carbonado_amd/lib"),
    };
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=carbonado_hip");
    // find the .so at run time without LD_LIBRARY_PATH
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
    println!("cargo:rerun-if-env-changed=CARBONADO_HIP_LIB_DIR");
    println!("cargo:rerun-if-changed=../include/carbonado_hip.h");
}
