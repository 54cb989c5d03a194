"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/pbft_verify.h declares, and fails loudly without a gfx950 GPU."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include")))
           if h.endswith(".h")]


def declared_functions():
    """Every function declared by include/*.h (pbft_verify.h, pbft_replica.h, pbft_wire.h)."""
    names = set()
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        src = re.sub(r"typedef[^;]*;", "", src)  # function-pointer typedefs are not exports
        # header-only helpers (static inline, e.g. pbft_votes_chunk_end) are not exports either; nor are the calls
        # inside their bodies or inside macros
        src = re.sub(r"static inline[^{]*\{.*?\n\}", "", src, flags=re.S)
        src = re.sub(r"#define[^\n]*(\\\n[^\n]*)*", "", src)
        names |= set(re.findall(r"\b(pbft_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_header_declares_expected_surface():
    fns = declared_functions()
    for f in ("pbft_verify_ctx_create", "pbft_verify_set_keys", "pbft_verify_batch", "pbft_verify_batch_async",
              "pbft_verify_wait", "pbft_verify_batch_device", "pbft_digest_blake2b512", "pbft_digest_sha256",
              "pbft_sign_batch", "pbft_verify_ctx_destroy"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    import pbft_amd
    lib = pbft_amd.load()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert set(declared_functions()) <= set(pbft_amd.EXPORTS) | set(declared_functions())
    assert b"gfx950" in lib.pbft_build_info()


def test_no_cpu_fallback_without_gpu():
    """On a host without a gfx950 GPU the product refuses to run (no silent CPU path)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import pbft_amd
    with pytest.raises(pbft_amd.PbftError) as e:
        pbft_amd.GpuBatchVerifier(0)
    assert e.value.code == -5  # PBFT_ENODEV


def test_null_arguments_are_errors_not_crashes():
    import pbft_amd
    lib = pbft_amd.load()
    assert lib.pbft_verify_ctx_create(0, None) == -1
    assert lib.pbft_verify_set_keys(None, None, 0, None) == -1
    assert lib.pbft_verify_batch(None, None, None, None, None, 0, 0, 0, None) == -1
    assert lib.pbft_verify_ctx_destroy(None) == 0
    assert lib.pbft_verify_update_keys(None, None, None, 0, None) == -1
    assert lib.pbft_verify_key_stats(None, None) == -1
