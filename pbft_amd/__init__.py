"""pbft_amd — MI355X-native batch Ed25519 verifier for PBFT prepare/commit quorums.

The product is the HIP/C++ library pbft_amd/libpbft_verify.so (C ABI in
include/pbft_verify.h).  This package is the thin host-side binding used by
tests and bench.py; it never computes a signature check itself.
"""
from ._lib import EXPORTS, LIB_PATH, PbftError, load  # noqa: F401
from .verifier import GpuBatchVerifier, MultiGpu, SigBatch, bitmap_to_bool, verify_multi  # noqa: F401

__all__ = ["GpuBatchVerifier", "MultiGpu", "SigBatch", "bitmap_to_bool", "verify_multi", "PbftError", "load", "LIB_PATH", "EXPORTS"]
