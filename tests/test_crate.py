"""The pbft-hip crate (pbft-hip/, Rust source; no Rust toolchain in this image, so it is not compiled here) must bind
exactly the C ABI the library exports: every function include/*.h declares appears in pbft-hip/src/ffi.rs with the
same number of parameters, and build.rs compiles the same sources for gfx950 as __graft_entry__.build()."""
import os
import re

from conftest import ROOT

CRATE = os.path.join(ROOT, "pbft-hip")


def _header_decls():
    out = {}
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if not h.endswith(".h"):
            continue
        src = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", h)).read(), flags=re.S)
        src = re.sub(r"typedef[^;]*;", "", src)
        src = re.sub(r"static inline[^{]*\{.*?\n\}", "", src, flags=re.S)  # header-only helpers: not exports
        src = re.sub(r"#define[^\n]*(\\\n[^\n]*)*", "", src)
        for m in re.finditer(r"\b(pbft_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
            args = m.group(2).strip()
            out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def _rust_decls():
    src = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    out = {}
    for m in re.finditer(r"pub fn (pbft_[a-z0-9_]+)\s*\((.*?)\)\s*(->[^;]*)?;", src, flags=re.S):
        args = m.group(2).strip().rstrip(",")
        out[m.group(1)] = 0 if not args else args.count(",") + 1
    return out


def test_ffi_binds_every_declared_function_with_its_arity():
    h, r = _header_decls(), _rust_decls()
    assert len(h) > 40
    missing = sorted(set(h) - set(r))
    extra = sorted(set(r) - set(h))
    assert not missing and not extra, (missing, extra)
    bad = {f: (h[f], r[f]) for f in h if h[f] != r[f]}
    assert not bad, bad


def test_build_rs_matches_graft_build():
    b = open(os.path.join(CRATE, "build.rs")).read()
    g = open(os.path.join(ROOT, "__graft_entry__.py")).read()
    for flag in ("--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared"):
        assert flag in b and flag in g, flag
    # the same translation units as pbft_amd/native_build.py (the product build), in the same roles
    import sys
    sys.path.insert(0, ROOT)
    from pbft_amd import native_build
    m = re.search(r"let hip_sources = \[([^\]]*)\]", b)
    assert m, "build.rs: hip_sources list not found"
    assert re.findall(r'"([^"]+)"', m.group(1)) == native_build.HIP_SOURCES
    m = re.search(r'for name in \[([^\]]*)\]\.iter\(\)', b)
    assert m, "build.rs: host source list not found"
    assert [x + ".cpp" for x in re.findall(r'"([^"]+)"', m.group(1))] == native_build.HOST_SOURCES
    for flag in native_build.HIP_FLAGS:
        assert flag in b, flag
    for flag in native_build.HOST_FLAGS:
        assert flag in b, flag
    assert 'links = "pbft_verify"' in open(os.path.join(CRATE, "Cargo.toml")).read()


def test_trait_surface():
    lib = open(os.path.join(CRATE, "src", "lib.rs")).read()
    for item in ("pub trait BatchVerifier", "fn submit(", "fn poll(", "fn verify(", "impl BatchVerifier for GpuVerifier",
                 "impl BatchVerifier for CpuVerifier", "verify_strict", "pub struct Replica", "fn key_from_peer_id",
                 "fn flush_submit(", "fn flush_poll(", "fn submit_votes(", "pub struct MultiGpu"):
        assert item in lib, item
