"""TEST INFRASTRUCTURE — NOT PRODUCT CODE.

Pure-Python CPU restatement of the Ed25519 verify/sign semantics on the PBFT
prepare/commit hot path.  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import this module, and only as the checker.

What it restates
----------------
The reference (ameya-deshmukh/pbft) carries no message signatures yet: the
signature checks are TODOs at `src/behavior.rs:127` (pre-prepare) and
`src/behavior.rs:185` (commit).  Its only Ed25519 code is the libp2p identity
key (`src/main.rs:39-40`), which reaches the curve arithmetic through third-party
crates that are NOT vendored under /root/reference:

  * libp2p 0.42.2 -> libp2p-core 0.31.1 identity::ed25519   (Cargo.lock:1295-1327)
  * ed25519-dalek 1.0.1  (`PublicKey::verify_strict`)          (Cargo.lock:668-679)
  * curve25519-dalek 3.2.1 (`CompressedEdwardsY::decompress`,
    `EdwardsPoint::is_small_order`, `Scalar::from_hash`,
    `vartime_double_scalar_mul_basepoint`)                      (Cargo.lock:604-614)
  * sha2 0.9.9 (SHA-512 inside verify)                          (Cargo.lock:2784-2787)
  * blake2 0.10.6 (request digest, `src/message.rs:209-212`)    (Cargo.lock:369-375)

The published algorithms restated here (semantics per SURVEY.md Appendix A):

  verify_strict(A_bytes, sig = R_bytes || s_bytes, M):
    1. s = LE(s_bytes); reject if s >= L            (ed25519-dalek check_scalar)
    2. A = decompress(A_bytes); reject on failure    (PublicKey::from_bytes)
    3. R = decompress(R_bytes); reject on failure
    4. reject if [8]R == O or [8]A == O              (is_small_order)
    5. k = SHA-512(R_bytes || A_bytes || M) mod L    (raw input bytes hashed)
    6. R' = [k](-A) + [s]B
    7. accept iff R' == R as group elements          (EdwardsPoint PartialEq)

  decompress(bytes) (curve25519-dalek 3.2.1):
    y = LE(bytes) with bit 255 cleared, NOT checked < p (reduced silently);
    (ok, x) = sqrt_ratio_i(y^2 - 1, d*y^2 + 1), x the non-negative root;
    reject if !ok; x = -x if sign bit set (x = 0 with sign 1 is accepted).

Parity pinning: RFC 8032 section 7.1 TEST 1-3 known answers (tests/golden),
RFC 7693 BLAKE2b KAT, and cross-checks against libsodium 1.0.18 / OpenSSL 3.0.2
on the vector classes where their semantics coincide with dalek verify_strict.
"""
from __future__ import annotations

import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

# Base point B = (x, 4/5)
_BY = (4 * pow(5, P - 2, P)) % P


def _is_negative(x: int) -> int:
    return (x % P) & 1


def sqrt_ratio_i(u: int, v: int):
    """curve25519-dalek 3.2.1 FieldElement::sqrt_ratio_i: returns (was_nonzero_square, r>=0).

    u == 0 -> (True, 0).  v == 0, u != 0 -> (False, 0).
    """
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = (u * v3 % P) * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct = check == u
    flipped = check == (-u) % P
    flipped_i = check == (-u * SQRT_M1) % P
    if flipped or flipped_i:
        r = r * SQRT_M1 % P
    if _is_negative(r):
        r = (-r) % P
    return (correct or flipped), r


def decompress(b: bytes):
    """CompressedEdwardsY::decompress -> extended point (X, Y, Z, T) or None."""
    assert len(b) == 32
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)
    y %= P  # FieldElement::from_bytes reduces silently (no canonicity check)
    yy = y * y % P
    u = (yy - 1) % P
    v = (yy * D + 1) % P
    ok, x = sqrt_ratio_i(u, v)
    if not ok:
        return None
    if b[31] >> 7:
        x = (-x) % P
    return (x, y, 1, x * y % P)


IDENT = (0, 1, 1, 0)


def pt_add(p, q):
    """Extended twisted-Edwards addition (a = -1), complete for d non-square."""
    x1, y1, z1, t1 = p
    x2, y2, z2, t2 = q
    a = (y1 - x1) * (y2 - x2) % P
    b = (y1 + x1) * (y2 + x2) % P
    c = t1 * D2 % P * t2 % P
    dd = 2 * z1 * z2 % P
    e, f, g, h = b - a, dd - c, dd + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def pt_neg(p):
    x, y, z, t = p
    return ((-x) % P, y, z, (-t) % P)


def pt_mul(k: int, p):
    q = IDENT
    while k > 0:
        if k & 1:
            q = pt_add(q, p)
        p = pt_add(p, p)
        k >>= 1
    return q


def pt_eq(p, q) -> bool:
    x1, y1, z1, _ = p
    x2, y2, z2, _ = q
    return (x1 * z2 - x2 * z1) % P == 0 and (y1 * z2 - y2 * z1) % P == 0


def is_identity(p) -> bool:
    return pt_eq(p, IDENT)


def is_small_order(p) -> bool:
    """EdwardsPoint::is_small_order: [8]P == identity."""
    q = p
    for _ in range(3):
        q = pt_add(q, q)
    return is_identity(q)


def compress(p) -> bytes:
    x, y, z, _ = p
    zi = pow(z, P - 2, P)
    x = x * zi % P
    y = y * zi % P
    return (y | (_is_negative(x) << 255)).to_bytes(32, "little")


BASE = decompress(_BY.to_bytes(32, "little"))  # sign bit 0: x is the even root


def sha512(data: bytes) -> bytes:
    return hashlib.sha512(data).digest()


def scalar_from_hash(h: bytes) -> int:
    """Scalar::from_hash: 64-byte digest, little-endian, reduced mod L."""
    return int.from_bytes(h, "little") % L


def verify_strict(pk: bytes, sig: bytes, msg: bytes) -> bool:
    """ed25519-dalek 1.0.1 PublicKey::verify_strict (see module docstring)."""
    if len(sig) != 64 or len(pk) != 32:
        return False
    s = int.from_bytes(sig[32:], "little")
    if s >= L:
        return False
    a = decompress(pk)
    if a is None:
        return False
    r = decompress(sig[:32])
    if r is None:
        return False
    if is_small_order(r) or is_small_order(a):
        return False
    k = scalar_from_hash(sha512(sig[:32] + pk + msg))
    rp = pt_add(pt_mul(k, pt_neg(a)), pt_mul(s, BASE))
    return pt_eq(rp, r)


def key_ok(pk: bytes) -> bool:
    """Key-table admission used by the batch verifier: decodes and is not small order.

    A key failing this makes every signature under it reject in verify_strict
    (steps 2 and 4), independent of R, s and M.
    """
    a = decompress(pk)
    return a is not None and not is_small_order(a)


# --- RFC 8032 signing (synthetic-data generation and KATs) -----------------

def secret_expand(seed: bytes):
    h = sha512(seed)
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, h[32:]


def public_key(seed: bytes) -> bytes:
    a, _ = secret_expand(seed)
    return compress(pt_mul(a, BASE))


def sign(seed: bytes, msg: bytes) -> bytes:
    a, prefix = secret_expand(seed)
    pk = compress(pt_mul(a, BASE))
    r = int.from_bytes(sha512(prefix + msg), "little") % L
    rb = compress(pt_mul(r, BASE))
    k = int.from_bytes(sha512(rb + pk + msg), "little") % L
    s = (r + k * a) % L
    return rb + s.to_bytes(32, "little")


# --- request digest (src/message.rs:209-212) --------------------------------

def request_digest(operation: bytes) -> bytes:
    """Blake2b-512 of the ClientRequest operation bytes (raw 64-byte digest)."""
    return hashlib.blake2b(operation, digest_size=64).digest()


def request_digest_hex(operation: bytes) -> str:
    """`digest()` at src/message.rs:209-212: `format!("{:x}", Blake2b::digest(m))`."""
    return request_digest(operation).hex()


def sha256(data: bytes) -> bytes:
    return hashlib.sha256(data).digest()
