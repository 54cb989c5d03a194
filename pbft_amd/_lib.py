"""ctypes binding of libpbft_verify.so (the C ABI in include/pbft_verify.h).

This is plumbing for tests and bench.py: the product is the HIP library.  There
is NO CPU fallback: if the in-tree shared library is missing, or no gfx950 GPU
is visible, every entry point raises PbftError.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PBFT_VERIFY_LIB") or os.path.join(_HERE, "libpbft_verify.so")  # override: A/B builds

# every symbol include/pbft_verify.h declares
EXPORTS = (
    "pbft_verify_ctx_create", "pbft_verify_ctx_destroy", "pbft_verify_ctx_clone", "pbft_verify_set_keys",
    "pbft_verify_update_keys", "pbft_verify_key_stats", "pbft_verify_revoke_keys", "pbft_verify_key_set_id",
    "pbft_verify_batch", "pbft_verify_batch_multi", "pbft_verify_batch_async", "pbft_verify_poll", "pbft_verify_wait",
    "pbft_verify_batch_device", "pbft_verify_reserve", "pbft_digest_blake2b512", "pbft_digest_sha256",
    "pbft_sign_batch", "pbft_last_error", "pbft_build_info", "pbft_last_kernel_ms", "pbft_verify_ctx_info",
    "pbft_verify_set_option", "pbft_verify_batch_device_pipelined", "pbft_verify_votes", "pbft_verify_votes_device",
    "pbft_verify_votes_async", "pbft_verify_votes_stage", "pbft_verify_votes_submit",
    "pbft_multi_create", "pbft_multi_destroy", "pbft_verify_batch_device_multi", "pbft_multi_sync",
    # include/pbft_wire.h
    "pbft_uvi_encode", "pbft_uvi_decode", "pbft_wire_encode_json", "pbft_wire_encode_frame",
    "pbft_wire_decode_json", "pbft_wire_decode_votes", "pbft_records_pack", "pbft_verify_records_device",
    "pbft_verify_records", "pbft_wire_encode_votes",
)

ERRORS = {0: "PBFT_OK", -1: "PBFT_EINVAL", -2: "PBFT_EHIP", -3: "PBFT_ENOKEYS",
          -4: "PBFT_ENOMEM", -5: "PBFT_ENODEV", -6: "PBFT_EBUSY"}


class PbftError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


_lib = None


def load() -> ctypes.CDLL:
    """Load the in-tree HIP library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so.7.
    # Importing torch first makes this library bind to that same runtime (same
    # SONAME), so torch tensors / streams and our contexts share one HIP
    # instance.  Loading ours first would pull /opt/rocm's copy and leave torch
    # unable to initialise.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise PbftError(-5, f"{LIB_PATH} not built: run python -c 'import __graft_entry__ as g; g.build()'")
    lib = ctypes.CDLL(LIB_PATH)
    vp, u8p = ctypes.c_void_p, ctypes.c_void_p
    i32, u32, u64 = ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64
    sig = {
        "pbft_verify_ctx_create": (i32, [i32, ctypes.POINTER(vp)]),
        "pbft_verify_ctx_destroy": (i32, [vp]),
        "pbft_verify_ctx_clone": (i32, [vp, ctypes.POINTER(vp)]),
        "pbft_verify_set_keys": (i32, [vp, u8p, u32, u8p]),
        "pbft_verify_update_keys": (i32, [vp, vp, u8p, u32, u8p]),
        "pbft_verify_key_stats": (i32, [vp, vp]),
        "pbft_verify_batch": (i32, [vp, u8p, u8p, vp, u8p, u32, u32, u64, vp]),
        "pbft_verify_batch_async": (i32, [vp, u8p, u8p, vp, u8p, u32, u32, u64, vp]),
        "pbft_verify_batch_multi": (i32, [vp, u32, u8p, u8p, vp, u8p, u32, u32, u64, vp]),
        "pbft_verify_poll": (i32, [vp]),
        "pbft_verify_wait": (i32, [vp]),
        "pbft_verify_batch_device": (i32, [vp, vp, vp, vp, vp, u32, u32, u64, vp, vp]),
        "pbft_verify_reserve": (i32, [vp, u64]),
        "pbft_digest_blake2b512": (i32, [vp, u8p, vp, vp, u64, u8p]),
        "pbft_digest_sha256": (i32, [vp, u8p, vp, vp, u64, u8p]),
        "pbft_sign_batch": (i32, [vp, u8p, u32, vp, u8p, u32, u32, u64, u8p, u8p, u8p]),
        "pbft_last_error": (ctypes.c_char_p, []),
        "pbft_build_info": (ctypes.c_char_p, []),
        "pbft_last_kernel_ms": (ctypes.c_float, [vp]),
        "pbft_verify_ctx_info": (i32, [vp, vp, vp, vp]),
        "pbft_verify_set_option": (i32, [vp, i32, u64]),
        "pbft_verify_batch_device_pipelined": (i32, [vp, vp, vp, vp, vp, u32, u32, u64, vp, vp, vp]),
        "pbft_verify_votes": (i32, [vp, vp, vp, vp, vp, vp, u32, u64, vp]),
        "pbft_verify_votes_device": (i32, [vp, vp, vp, vp, vp, vp, u32, u64, vp, vp]),
        "pbft_verify_votes_async": (i32, [vp, vp, vp, vp, vp, vp, u32, u64, vp]),
        "pbft_verify_votes_stage": (i32, [vp, u64, u32, vp]),
        "pbft_verify_votes_submit": (i32, [vp, u64, u32, vp]),
        "pbft_verify_votes_submit_begin": (i32, [vp, u64, u32, vp]),
        "pbft_verify_votes_submit_rows": (i32, [vp, u64]),
        "pbft_verify_poll_rows": (i32, [vp, ctypes.POINTER(u64)]),
        "pbft_verify_votes_submit_host": (i32, [vp, vp, u64, vp, u32, vp]),
        "pbft_host_alloc": (i32, [vp, ctypes.c_size_t, ctypes.POINTER(vp)]),
        "pbft_verify_votes_open": (i32, [vp, u64, u32, vp]),
        "pbft_verify_votes_piece": (i32, [vp, vp, u64, u64, vp, u32, u32]),
        "pbft_verify_votes_close": (i32, [vp, u64]),
        "pbft_host_free": (i32, [vp, vp]),
        "pbft_multi_create": (i32, [vp, u32, ctypes.POINTER(vp)]),
        "pbft_multi_destroy": (i32, [vp]),
        "pbft_multi_sync": (i32, [vp]),
        "pbft_verify_batch_device_multi": (i32, [vp, vp, vp, vp, vp, u32, u32, vp, u64, vp]),
        "pbft_uvi_encode": (ctypes.c_size_t, [u64, u8p]),
        "pbft_uvi_decode": (i32, [u8p, ctypes.c_size_t, vp, vp]),
        "pbft_wire_encode_json": (i32, [vp, vp, ctypes.c_size_t, vp]),
        "pbft_wire_encode_frame": (i32, [vp, vp, ctypes.c_size_t, vp]),
        "pbft_wire_decode_json": (i32, [vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t]),
        "pbft_wire_decode_votes": (i32, [u8p, ctypes.c_size_t, u32, u64, u64, vp, vp, vp, vp, vp, vp, vp, vp,
                                         vp, vp, vp]),
        "pbft_records_pack": (i32, [vp, vp, vp, vp, u32, u64, vp]),
        "pbft_wire_encode_votes": (i32, [u64, vp, vp, vp, vp, vp, vp, vp, ctypes.c_size_t, vp]),
        "pbft_verify_revoke_keys": (i32, [vp, vp, u32]),
        "pbft_verify_key_set_id": (i32, [vp, ctypes.POINTER(u64)]),
        "pbft_verify_records_device": (i32, [vp, vp, u64, vp, vp]),
        "pbft_verify_records": (i32, [vp, vp, u64, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int) -> int:
    if rc < 0:
        raise PbftError(rc, load().pbft_last_error().decode(errors="replace"))
    return rc
