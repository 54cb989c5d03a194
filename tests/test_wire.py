"""Wire codec (include/pbft_wire.h) — CPU tests, no GPU needed.

Oracle: Python's json.dumps(obj, separators=(",", ":"), ensure_ascii=False) is
byte-identical to serde_json::to_string for these structs (same field order,
same escapes), which is what the reference sends (message_to_json,
src/protocol_config.rs:116-123).  Varint vectors follow the unsigned-varint /
LEB128 spec used by UviBytes (src/protocol_config.rs:51, :82).  The one
message the reference itself holds is the client request in README.md:42.
"""
import hashlib
import json
import random

import numpy as np
import pytest

from pbft_amd import wire
from pbft_amd.wire import COMMIT, CLIENT_REQUEST, PREPARE, PREPREPARE, WireMsg

README_REQUEST = b'{"ClientRequest": {"operation": "testOperation", "timestamp": 1, "client": "127.0.0.1:9000"}}'


def ref_json(kind, view=0, seq=0, digest=bytes(64), replica=None, sig=None, op=b"", ts=0, client=""):
    """The reference's serde_json bytes (plus the signed-envelope fields when present)."""
    cr = {"operation": op.decode(), "timestamp": ts, "client": client}
    if kind == CLIENT_REQUEST:
        obj = {"ClientRequest": cr}
    else:
        body = {"view": view, "sequence_number": seq, "digest": digest.hex()}
        if kind == PREPREPARE:
            body["message"] = cr
        if sig is not None:
            body["replica"] = replica
            body["signature"] = sig.hex()
        obj = {["PrePrepare", "Prepare", "Commit"][kind]: body}
    return json.dumps(obj, separators=(",", ":"), ensure_ascii=False).encode()


@pytest.mark.parametrize("v,enc", [(0, "00"), (1, "01"), (127, "7f"), (128, "8001"), (255, "ff01"), (300, "ac02"),
                                   (16384, "808001"), (2**32, "8080808010"), (2**64 - 1, "ffffffffffffffffff01")])
def test_uvi_vectors(v, enc):
    assert wire.uvi_encode(v).hex() == enc
    assert wire.uvi_decode(bytes.fromhex(enc) + b"\xaa") == (v, len(enc) // 2)


def test_uvi_rejects_and_partial():
    assert wire.uvi_decode(b"\x80") is None            # need more bytes
    assert wire.uvi_decode(b"") is None
    for bad in ("8000", "ff00", "ffffffffffffffffff02", "ffffffffffffffffffff01"):
        with pytest.raises(Exception):
            wire.uvi_decode(bytes.fromhex(bad))


def test_readme_client_request_round_trip():
    m = wire.decode_json(README_REQUEST)
    assert (m.kind, m.operation, m.timestamp, m.client) == (CLIENT_REQUEST, b"testOperation", 1, "127.0.0.1:9000")
    assert wire.encode_json(m) == ref_json(CLIENT_REQUEST, op=b"testOperation", ts=1, client="127.0.0.1:9000")


OPS = [b"testOperation", b"", b'quote " backslash \\ slash /', b"ctl \x00\x01\x08\x09\x0a\x0c\x0d\x1f\x7f",
       "unicode é ✓ 𝄞".encode(), bytes(range(0x20, 0x7f))]


@pytest.mark.parametrize("op", OPS)
def test_encode_matches_serde_json(op):
    rnd = random.Random(len(op))
    d = hashlib.blake2b(op, digest_size=64).digest()
    sig = bytes(rnd.randrange(256) for _ in range(64))
    for kind in (PREPREPARE, PREPARE, COMMIT, CLIENT_REQUEST):
        for signed in (False, True):
            if kind == CLIENT_REQUEST and signed:
                continue
            m = WireMsg(kind=kind, view=2**64 - 1 if signed else 0, seq=12345, digest=d,
                        replica=7 if signed else None, sig=sig if signed else None, operation=op,
                        timestamp=1700000000, client="[::1]:9000")
            want = ref_json(kind, m.view, m.seq, d, m.replica, m.sig, op, m.timestamp, m.client)
            got = wire.encode_json(m)
            assert got == want
            back = wire.decode_json(got)
            cr = kind == CLIENT_REQUEST  # a ClientRequest carries no view / seq / digest
            assert (back.kind, back.view, back.seq, back.digest, back.replica, back.sig) == \
                (kind, 0 if cr else m.view, 0 if cr else m.seq, bytes(64) if cr else d, m.replica, m.sig)
            if kind in (PREPREPARE, CLIENT_REQUEST):
                assert (back.operation, back.timestamp, back.client) == (op, m.timestamp, m.client)
            frame = wire.encode_frame(m)
            assert frame == wire.uvi_encode(len(want)) + want


def test_decoder_accepts_what_serde_accepts():
    d = bytes(range(64)).hex()
    pretty = ('{ "Prepare" : {\n  "digest": "%s",\n  "extra": [1, {"a": null}, true, -2.5e3],\n'
              '  "sequence_number" : 9 ,"view":0 } }\n' % d).encode()
    m = wire.decode_json(pretty)
    assert (m.kind, m.view, m.seq, m.digest.hex()) == (PREPARE, 0, 9, d)
    esc = b'{"ClientRequest":{"operation":"a\\u00e9\\ud834\\udd1e\\/\\n","timestamp":0,"client":"1.2.3.4:5"}}'
    assert wire.decode_json(esc).operation == "aé𝄞/\n".encode()
    # non-hex / uppercase digest: a valid Message, but no binary envelope
    up = b'{"Commit":{"view":1,"sequence_number":2,"digest":"%s"}}' % bytes(range(64)).hex().upper().encode()
    assert wire.decode_json(up).digest_ok is False


def test_decoder_fast_paths_match_the_escaped_forms():
    """r06: strings without escapes are read in place (keys, hex digest / signature: 8 characters per step); an
    escaped spelling of the same text must decode the same, and one wrong character anywhere must be caught."""
    d = bytes(range(64)).hex()
    plain = b'{"Commit":{"view":3,"sequence_number":7,"digest":"%s"}}' % d.encode()
    # the same JSON text with the key and some digest characters written as \\u escapes
    esc_d = "".join("\\u%04x" % ord(c) if i % 5 == 0 else c for i, c in enumerate(d))
    escaped = b'{"Commit":{"vi\\u0065w":3,"sequence_number":7,"digest":"%s"}}' % esc_d.encode()
    for js in (plain, escaped):
        m = wire.decode_json(js)
        assert (m.kind, m.view, m.seq, m.digest_ok, m.digest.hex()) == (COMMIT, 3, 7, True, d)
    for pos in (0, 1, 7, 8, 63, 64, 120, 127):
        for c in "gG/:`{AF\x7f":
            bad_d = d[:pos] + c + d[pos + 1:]
            js = b'{"Commit":{"view":3,"sequence_number":7,"digest":"%s"}}' % bad_d.encode()
            assert wire.decode_json(js).digest_ok is False, (pos, c)


def _decode_or_err(js):
    try:
        m = wire.decode_json(js)
    except Exception as e:  # noqa: BLE001 -- the error itself is what is compared
        return ("err", getattr(e, "code", None))
    return (m.kind, m.view, m.seq, m.digest, m.digest_ok, m.replica, m.sig, m.operation, m.timestamp, m.client)


def test_canonical_vote_fast_path_equals_general_parser():
    """r06: a signed vote in serde's exact compact form is matched byte for byte (fast_vote); with one space added
    after every ':' the general parser decodes the same message.  Both must agree on every field, and on the
    near-canonical inputs that the fast path hands back (bad numbers, hex, trailing bytes, other fields)."""
    rnd = random.Random(6)
    for i in range(300):
        kind = rnd.choice([PREPARE, COMMIT])
        m = WireMsg(kind=kind, view=rnd.choice([0, 1, 9, 10, 2**63, 2**64 - 1, rnd.randrange(2**64)]),
                    seq=rnd.randrange(2**64), digest=bytes(rnd.randrange(256) for _ in range(64)),
                    replica=rnd.choice([0, 1, 255, 65535, rnd.randrange(65536)]),
                    sig=bytes(rnd.randrange(256) for _ in range(64)))
        compact = wire.encode_json(m)
        spaced = compact.replace(b'":', b'": ')
        assert compact != spaced
        a, b = _decode_or_err(compact), _decode_or_err(spaced)
        assert a == b and a[0] == kind, (compact, a, b)
    d, sg = bytes(range(64)).hex(), bytes(range(64, 128)).hex()
    base = '{"Prepare":{"view":%s,"sequence_number":%s,"digest":"%s","replica":%s,"signature":"%s"}}'
    cases = [("1", "2", d, "3", sg), ("01", "2", d, "3", sg), ("0", "00", d, "3", sg),
             ("18446744073709551615", "2", d, "3", sg), ("18446744073709551616", "2", d, "3", sg),
             ("1", "2", d.upper(), "3", sg), ("1", "2", d[:-1] + "g", "3", sg), ("1", "2", d, "65535", sg),
             ("1", "2", d, "65536", sg), ("1", "2", d, "3", sg[:-2]), ("1", "2", d, "3", sg + "00"),
             ("1.0", "2", d, "3", sg), ("1", "2e3", d, "3", sg), ("-1", "2", d, "3", sg), ("1", "2", d, "3", "zz" * 64)]
    for c in cases:
        compact = (base % c).encode()
        spaced = compact.replace(b'":', b'": ')
        assert _decode_or_err(compact) == _decode_or_err(spaced), (c, _decode_or_err(compact))
    # trailing bytes, an extra field, a different field order: only the general parser can say (same answers)
    tail = (base % ("1", "2", d, "3", sg)).encode()
    for js in (tail + b" ", tail + b"x", tail[:-2] + b',"extra":null}}',
               b'{"Prepare":{"sequence_number":2,"view":1,"digest":"%s","replica":3,"signature":"%s"}}' % (
                   d.encode(), sg.encode())):
        got = _decode_or_err(js)
        assert got == _decode_or_err(js.replace(b'":', b'": ')), js
    assert _decode_or_err(tail + b" ")[0] == PREPARE and _decode_or_err(tail + b"x")[0] == "err"


@pytest.mark.parametrize("bad", [
    b'{"Prepare":{"view":1,"sequence_number":2}}',                                   # missing digest
    b'{"Prepare":{"view":1,"view":1,"sequence_number":2,"digest":""}}',              # duplicate field
    b'{"Prepare":{"view":01,"sequence_number":2,"digest":""}}',                      # leading zero
    b'{"Prepare":{"view":1.0,"sequence_number":2,"digest":""}}',                     # float
    b'{"Prepare":{"view":-1,"sequence_number":2,"digest":""}}',                      # negative
    b'{"Prepare":{"view":18446744073709551616,"sequence_number":2,"digest":""}}',    # > u64
    b'{"Prepare":{"view":1,"sequence_number":2,"digest":""}} x',                     # trailing
    b'{"Vote":{"view":1,"sequence_number":2,"digest":""}}',                          # unknown variant
    b'{"Prepare":{"view":1,"sequence_number":2,"digest":"\\ud800"}}',                 # lone surrogate
    b'{"Prepare":{"view":1,"sequence_number":2,"digest":"\xff"}}',                   # invalid UTF-8
    b'{"Prepare":{"view":1,"sequence_number":2,"digest":"a\x01"}}',                  # raw control char
    b'{"Prepare":{"view":1,"sequence_number":2,"digest":"","replica":1}}',           # half an extension
    b'{"PrePrepare":{"view":1,"sequence_number":2,"digest":""}}',                    # missing message
    b'{"Prepare":{"view":1,"sequence_number":2,"digest":"","replica":70000,"signature":""}}',
    b'',
])
def test_decoder_rejects_what_serde_rejects(bad):
    with pytest.raises(Exception):
        wire.decode_json(bad)


def envelope(kind, view, seq, digest):
    return b"PBFT" + bytes([kind]) + view.to_bytes(8, "little") + seq.to_bytes(8, "little") + digest


def test_decode_votes_stream_to_soa():
    rnd = random.Random(5)
    frames, exp_status, exp_rows = [], [], []
    for i in range(300):
        kind = rnd.choice([PREPARE, COMMIT])
        d = hashlib.blake2b(b"op-%d" % i, digest_size=64).digest()
        sig = bytes(rnd.randrange(256) for _ in range(64))
        m = WireMsg(kind=kind, view=rnd.randrange(4), seq=i, digest=d, replica=rnd.randrange(6), sig=sig)
        st = 0
        r = rnd.random()
        if r < 0.1:
            m.sig, m.replica, st = None, None, 3                     # unsigned (reference-format) vote
        elif r < 0.15:
            m.kind, m.operation, m.client, st = PREPREPARE, b"x", "1.1.1.1:1", 0  # signed PrePrepare: kind-0 row
        elif r < 0.17:
            m = WireMsg(kind=CLIENT_REQUEST, operation=b"op", timestamp=3, client="1.1.1.1:1")
            st = 4                                                    # not a replica-signed message
        elif r < 0.2:
            st = 5 if m.replica >= 4 else 0                           # n_replicas = 4 below
        frame = wire.encode_frame(m)
        if rnd.random() < 0.05:
            frame = wire.uvi_encode(5) + b"{oops"
            st = 1
        frames.append(frame)
        if st == 0 and m.replica is not None and m.replica >= 4:
            st = 5
        exp_status.append(st)
        if st == 0:
            exp_rows.append((m.sig, m.replica, envelope(m.kind, m.view, m.seq, d), m.kind, m.view, m.seq))
    stream = b"".join(frames)
    partial = wire.encode_frame(WireMsg(kind=PREPARE, view=1, seq=1, digest=bytes(64), replica=0, sig=bytes(64)))
    v = wire.decode_votes(stream + partial[:-3], n_replicas=4)
    assert v.consumed == len(stream)                                  # trailing partial frame kept back
    assert list(v.status) == exp_status
    assert len(v.R) == len(exp_rows)
    for i, (sig, rep, env, kind, view, seq) in enumerate(exp_rows):
        assert bytes(v.R[i]) + bytes(v.S[i]) == sig
        assert int(v.key_idx[i]) == rep and bytes(v.msg[i]) == env
        assert (int(v.kind[i]), int(v.view[i]), int(v.seq[i])) == (kind, view, seq)
    # resuming from `consumed` with the rest of the frame completes it
    v2 = wire.decode_votes(partial, n_replicas=4)
    assert list(v2.status) == [0] and v2.consumed == len(partial)


def test_decode_votes_framing_error():
    with pytest.raises(Exception):
        wire.decode_votes(bytes.fromhex("8000") + b"{}", n_replicas=4)


def test_records_pack_layout():
    rnd = np.random.default_rng(1)
    n = 37
    R, S = rnd.integers(0, 256, (n, 32), np.uint8), rnd.integers(0, 256, (n, 32), np.uint8)
    K = rnd.integers(0, 65536, n).astype(np.uint16)
    M = rnd.integers(0, 256, (n, 90), np.uint8)
    rec = wire.records_pack(R, S, K, M, 90)
    assert rec.shape == (n, 160)
    assert (rec[:, :32] == R).all() and (rec[:, 32:64] == S).all() and (rec[:, 64:149] == M[:, :85]).all()
    assert (rec[:, 150].astype(np.uint16) | (rec[:, 151].astype(np.uint16) << 8) == K).all()
    assert (rec[:, 149] == 0).all() and (rec[:, 152:] == 0).all()
