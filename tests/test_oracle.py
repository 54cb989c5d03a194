"""Pin the oracle: KATs, golden vectors, C vs Python restatement, libsodium / OpenSSL.

The reference has no tests and its Ed25519 arithmetic lives in
un-vendored crates (ed25519-dalek 1.0.1 / curve25519-dalek 3.2.1), so the
oracle is pinned by (1) RFC 8032 §7.1 known answers, (2) the RFC 7693 BLAKE2b
KAT and the request digest of the reference README's operation
(README.md:42, src/message.rs:209-212), (3) agreement of two independent
restatements (pure Python big-int, C radix-2^51), and (4) libsodium 1.0.18 and
OpenSSL 3.0.2 on the vector classes where their semantics equal dalek
verify_strict.
"""
import ctypes
import ctypes.util
import json
import os

import numpy as np
import pytest

import ed25519_ref as E
from conftest import GOLDEN, ROOT, golden_batches

KAT = json.load(open(os.path.join(GOLDEN, "kat.json")))


@pytest.fixture(scope="module")
def coracle():
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        os.system(f"make -s -C {os.path.join(ROOT, 'oracle')}")
    lib = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    lib.oracle_verify_strict.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    lib.oracle_verify_batch.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint64, vp, ctypes.c_int]
    lib.oracle_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    lib.oracle_public_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.oracle_key_ok.argtypes = [ctypes.c_char_p]
    return lib


# RFC 8032 §7.1 TEST 1-3 as published (hex), independent of our generator
RFC8032 = [
    ("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
     "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46b"
     "d25bf5f0595bbe24655141438e7a100b"),
    ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
     "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c"
     "387b2eaeb4302aeeb00d291612bb0c00"),
    ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
     "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
     "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc659"
     "4a7c15e9716ed28dc027beceea1ec40a"),
]


@pytest.mark.parametrize("sk,pk,msg,sig", RFC8032)
def test_rfc8032_python(sk, pk, msg, sig):
    seed, m = bytes.fromhex(sk), bytes.fromhex(msg)
    assert E.public_key(seed).hex() == pk
    assert E.sign(seed, m).hex() == sig
    assert E.verify_strict(bytes.fromhex(pk), bytes.fromhex(sig), m)


@pytest.mark.parametrize("sk,pk,msg,sig", RFC8032)
def test_rfc8032_c(coracle, sk, pk, msg, sig):
    seed, m = bytes.fromhex(sk), bytes.fromhex(msg)
    out = ctypes.create_string_buffer(32)
    coracle.oracle_public_key(out, seed)
    assert out.raw.hex() == pk
    so = ctypes.create_string_buffer(64)
    coracle.oracle_sign(so, seed, m, len(m))
    assert so.raw.hex() == sig
    assert coracle.oracle_verify_strict(bytes.fromhex(pk), bytes.fromhex(sig), m, len(m)) == 1


def test_kat_json_matches_rfc():
    got = {(t["secret"], t["public"], t["message"], t["signature"]) for t in KAT["rfc8032"]}
    assert got == set(RFC8032)


def test_request_digest_kats():
    # digest("testOperation") per src/message.rs:209-212
    assert E.request_digest_hex(b"testOperation") == (
        "292b3560871b52680690991f5077a31e687b1c0309fb796292ccf3e050d9ee0b"
        "6c644a02aa93b92c956c6c4442908afe34b7adb6e9969ae9b3f8e022af50cf69")
    assert E.sha256(b"testOperation").hex() == "e6ac89915f600c54dde6cae384fcf86b73501a05c6aa6bfae9c4811aefe0e27b"
    # RFC 7693 Appendix A: BLAKE2b-512("abc")
    assert E.request_digest(b"abc").hex().startswith("ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1")
    assert KAT["digest"]["blake2b512_hex"] == E.request_digest_hex(b"testOperation")


def test_small_order_and_noncanonical_tables():
    so = [bytes.fromhex(h) for h in KAT["small_order_encodings"]]
    assert len(so) == 14
    for b in so:
        p = E.decompress(b)
        assert p is not None and E.is_small_order(p)
    for h in KAT["noncanonical_decodable_encodings"]:
        b = bytes.fromhex(h)
        assert int.from_bytes(b, "little") & ((1 << 255) - 1) >= E.P
        assert E.decompress(b) is not None


def test_golden_expected_is_python_oracle(golden):
    """Spot-check that the committed expected bits are the Python oracle's (regenerable)."""
    for ml, b in golden_batches(golden):
        keys = b["keys"]
        for i in range(0, len(b["R"]), 37):
            pk = keys[b["key_idx"][i]].tobytes()
            sig = b["R"][i].tobytes() + b["S"][i].tobytes()
            m = b["msg"][i, :ml].tobytes()
            assert E.verify_strict(pk, sig, m) == bool(b["expected"][i]), (ml, i, int(b["cls"][i]))
        for j, k in enumerate(keys):
            assert E.key_ok(k.tobytes()) == bool(b["key_ok"][j])


def test_golden_class_coverage(golden):
    b = dict(golden_batches(golden))[85]
    cls, exp = b["cls"], b["expected"]
    assert set(cls.tolist()) >= set(range(18)) | {19}
    assert exp[cls == 0].all() and exp[cls == 18].all() and exp[cls == 10].all()  # valid + mixed-order accept
    for c in list(range(1, 18)) + [19]:
        if c != 10:
            assert not exp[cls == c].any(), c


def test_c_oracle_matches_golden(coracle, golden):
    for ml, b in golden_batches(golden):
        n = len(b["R"])
        out = np.zeros(n, dtype=np.uint8)
        msg = np.ascontiguousarray(b["msg"])
        assert coracle.oracle_verify_batch(b["keys"].ctypes.data, len(b["keys"]), b["R"].ctypes.data,
                                           b["S"].ctypes.data, b["key_idx"].ctypes.data, msg.ctypes.data, ml,
                                           msg.shape[1], n, out.ctypes.data, 4) == 0
        assert (out == b["expected"]).all(), (ml, np.nonzero(out != b["expected"])[0][:10])
        for j, k in enumerate(b["keys"]):
            assert coracle.oracle_key_ok(k.tobytes()) == b["key_ok"][j]


# --- third-party cross-checks (skipped where the library is absent) ---------

def _sodium():
    for p in ("/opt/conda/lib/libsodium.so.23", ctypes.util.find_library("sodium")):
        if p:
            try:
                lib = ctypes.CDLL(p)
                lib.sodium_init()
                return lib
            except OSError:
                pass
    return None


# classes where libsodium 1.0.18's verify_detached == dalek verify_strict
SODIUM_AGREES = {0, 1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13, 14, 16, 17, 18, 19}


def test_libsodium_agrees_on_its_classes(golden):
    lib = _sodium()
    if lib is None:
        pytest.skip("libsodium not present")
    f = lib.crypto_sign_ed25519_verify_detached
    f.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulonglong, ctypes.c_char_p]
    checked = 0
    for ml, b in golden_batches(golden):
        for i in range(len(b["R"])):
            c = int(b["cls"][i])
            if c not in SODIUM_AGREES:
                continue
            sig = b["R"][i].tobytes() + b["S"][i].tobytes()
            m = b["msg"][i, :ml].tobytes()
            pk = b["keys"][b["key_idx"][i]].tobytes()
            assert (f(sig, m, len(m), pk) == 0) == bool(b["expected"][i]), (ml, i, c)
            checked += 1
    assert checked > 1000


# classes without small-order/torsion points or non-canonical encodings: OpenSSL == dalek
OPENSSL_AGREES = {0, 1, 2, 3, 4, 5, 6, 11, 16, 17, 18, 19}


def test_openssl_agrees_on_its_classes(golden):
    path = ctypes.util.find_library("crypto")
    if not path:
        pytest.skip("libcrypto not present")
    L = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    L.EVP_PKEY_new_raw_public_key.restype = vp
    L.EVP_PKEY_new_raw_public_key.argtypes = [ctypes.c_int, vp, ctypes.c_char_p, ctypes.c_size_t]
    L.EVP_MD_CTX_new.restype = vp
    L.EVP_MD_CTX_free.argtypes = [vp]
    L.EVP_PKEY_free.argtypes = [vp]
    L.EVP_DigestVerifyInit.argtypes = [vp, vp, vp, vp, vp]
    L.EVP_DigestVerify.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
    NID_ED25519 = 1087
    checked = 0
    for ml, b in golden_batches(golden):
        for i in range(0, len(b["R"]), 3):
            c = int(b["cls"][i])
            if c not in OPENSSL_AGREES:
                continue
            pkb = b["keys"][b["key_idx"][i]].tobytes()
            pkey = L.EVP_PKEY_new_raw_public_key(NID_ED25519, None, pkb, 32)
            if not pkey:
                assert not b["expected"][i]
                continue
            ctx = L.EVP_MD_CTX_new()
            L.EVP_DigestVerifyInit(ctx, None, None, None, pkey)
            sig = b["R"][i].tobytes() + b["S"][i].tobytes()
            m = b["msg"][i, :ml].tobytes()
            rc = L.EVP_DigestVerify(ctx, sig, 64, m, len(m))
            L.EVP_MD_CTX_free(ctx)
            L.EVP_PKEY_free(pkey)
            assert (rc == 1) == bool(b["expected"][i]), (ml, i, c)
            checked += 1
    assert checked > 300


def test_fullround_special_key_construction(coracle):
    """tests/fullround.py (the builder of the GPU full-round parity test): a small-order key slot and a mixed-order
    key slot in the key set; Python-built equation-valid mixed-order signatures accept and cofactored-only ones
    reject, in both restatements (the C oracle is the GPU test's checker at 2^20 lanes)."""
    import fullround as F
    seeds = np.stack([np.frombuffer(bytes([i + 1]) * 32, np.uint8) for i in range(4)])
    pub = np.stack([np.frombuffer(E.public_key(s.tobytes()), np.uint8) for s in seeds])
    pub2, a = F.install_special_keys(seeds, pub, small_slot=2, mixed_slot=3)
    assert not E.key_ok(pub2[2].tobytes()) and E.key_ok(pub2[3].tobytes())
    n = 24
    key_idx = np.array([i % 4 for i in range(n)], np.uint16)
    msg = np.stack([np.frombuffer(b"PBFT" + bytes([1]) + (1).to_bytes(8, "little") + i.to_bytes(8, "little")
                                  + bytes(64), np.uint8) for i in range(n)])
    sigs = [E.sign(seeds[k].tobytes(), msg[i].tobytes()) for i, k in enumerate(key_idx)]
    R = np.stack([np.frombuffer(s[:32], np.uint8) for s in sigs])
    S = np.stack([np.frombuffer(s[32:], np.uint8) for s in sigs])
    R2, S2, v, c = F.plant_mixed(R, S, key_idx, msg, 85, pub2, a, 3, n_valid=3, n_cofactored=2, seed=7)
    assert len(v) == 3 and len(c) == 2
    exp = np.array([E.verify_strict(pub2[k].tobytes(), R2[i].tobytes() + S2[i].tobytes(), msg[i].tobytes())
                    for i, k in enumerate(key_idx)])
    out = np.zeros(n, np.uint8)
    assert coracle.oracle_verify_batch(pub2.ctypes.data, 4, R2.ctypes.data, S2.ctypes.data, key_idx.ctypes.data,
                                       np.ascontiguousarray(msg).ctypes.data, 85, 85, n, out.ctypes.data, 2) == 0
    assert (out.astype(bool) == exp).all()
    assert exp[v].all() and not exp[c].any()
    assert not exp[key_idx == 2].any()                        # small-order key: everything rejects
    planted = np.zeros(n, bool)
    planted[v] = planted[c] = True
    assert not exp[(key_idx == 3) & ~planted].any()           # signatures over the old key bytes reject under A'
    assert exp[(key_idx < 2)].all()
