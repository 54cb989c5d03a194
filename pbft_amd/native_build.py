"""Build of libpbft_verify.so (gfx950): the single place that lists the native sources and compiler lines.

Used by __graft_entry__.build() (the product library, in-tree) and tools/build_variant.py (A/B variants under
build/ab/).  The HIP sources compile to objects in parallel -- the four key plans' verify kernels live in their own
translation units (comb_pa*.hip) -- and are linked with the host-side state machine and wire codec.
pbft-hip/build.rs runs the same compiler lines.
"""
from __future__ import annotations

import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pbft_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_SOURCES = ["pbft_verify.hip", "tables.hip", "finish.hip", "sign.hip", "comb_pa13.hip", "comb_pa14.hip", "comb_pa16.hip", "comb_pa32.hip"]
HOST_SOURCES = ["replica.cpp", "wire.cpp"]
HIP_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall"]
HOST_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wextra"]
LIB = os.path.join(ROOT, "pbft_amd", "libpbft_verify.so")


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, cwd=ROOT, check=True)


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return hs + [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def build_library(out: str = LIB, defines=(), objdir: str | None = None, jobs: int = 8) -> str:
    """Compile (what is stale) and link `out`; `defines` are extra -D flags for an A/B variant."""
    objdir = objdir or os.path.join(ROOT, "build", "obj")
    os.makedirs(objdir, exist_ok=True)
    stamp = os.path.join(objdir, "defines.txt")
    want = " ".join(defines)
    if not os.path.exists(stamp) or open(stamp).read() != want:
        for f in os.listdir(objdir):
            if f.endswith(".o"):
                os.remove(os.path.join(objdir, f))
        with open(stamp, "w") as fh:
            fh.write(want)
    hdrs = _headers()
    host_objs, hip_objs, todo = [], [], []
    for src in HOST_SOURCES:
        s = os.path.join(CSRC, "host", src)
        o = os.path.join(objdir, src.replace(".cpp", ".o"))
        host_objs.append(o)
        if _stale(o, [s] + hdrs):
            todo.append(["g++"] + HOST_FLAGS + ["-c", "-o", o, s])
    for src in HIP_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(objdir, src.replace(".hip", ".o"))
        hip_objs.append(o)
        if _stale(o, [s] + hdrs):
            todo.append([HIPCC] + HIP_FLAGS + list(defines) + ["-c", "-o", o, s])
    # longest first
    todo.sort(key=lambda c: 0 if ("tables" in c[-1] or "pbft_verify" in c[-1]) else 1)
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, c) for c in todo]:
            f.result()
    objs = hip_objs + host_objs
    if todo or _stale(out, objs):
        _run([HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-Wl,-soname,libpbft_verify.so", "-o", out] + objs)
    return out


INGRESS_SRC = os.path.join(ROOT, "tools", "ingress", "ingress_driver.cpp")
INGRESS_LIB = os.path.join(ROOT, "tools", "ingress", "libingress.so")


def build_ingress_driver() -> str:
    """Bench infrastructure: the single-threaded ingress loops of bench.py's replica_ingress leg
    (tools/ingress/ingress_driver.cpp), linked against the in-tree library."""
    if _stale(INGRESS_LIB, [INGRESS_SRC, LIB] + _headers()):
        _run(["g++"] + HOST_FLAGS + ["-shared", "-o", INGRESS_LIB, INGRESS_SRC, "-L" + os.path.dirname(LIB),
                                     "-lpbft_verify", "-Wl,-rpath,$ORIGIN/../../pbft_amd"])
    return INGRESS_LIB
