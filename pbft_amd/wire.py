"""ctypes binding of the wire codec (include/pbft_wire.h, pbft_amd/csrc/host/wire.cpp).

Plumbing for tests and tools: UviBytes framing + serde_json Message encoding of
the reference (src/protocol_config.rs:41-129, src/message.rs:7-31) with the
signed-envelope fields, and the stream -> struct-of-arrays vote decoder that
feeds the GPU verifier.  The codec itself is the C++ library code.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from ._lib import PbftError, check, load

PREPREPARE, PREPARE, COMMIT, CLIENT_REQUEST = 0, 1, 2, 3
RECORD_BYTES = 160
ENVELOPE = 85
STATUS = {0: "ok", 1: "json", 2: "digest", 3: "unsigned", 4: "kind", 5: "signer"}


class _Msg(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("view", ctypes.c_uint64), ("seq", ctypes.c_uint64),
                ("digest", ctypes.c_uint8 * 64), ("digest_ok", ctypes.c_uint32), ("has_sig", ctypes.c_uint32),
                ("replica", ctypes.c_uint32), ("sig", ctypes.c_uint8 * 64), ("operation", ctypes.c_void_p),
                ("operation_len", ctypes.c_uint32), ("timestamp", ctypes.c_uint64), ("client", ctypes.c_char * 64)]


@dataclass
class WireMsg:
    kind: int
    view: int = 0
    seq: int = 0
    digest: bytes = bytes(64)
    replica: int | None = None      # signed-envelope extension
    sig: bytes | None = None        # R || S
    operation: bytes = b""          # ClientRequest (standalone or inside PrePrepare)
    timestamp: int = 0
    client: str = ""
    digest_ok: bool = True
    _keep: list = field(default_factory=list, repr=False)

    def _to_c(self) -> _Msg:
        m = _Msg()
        m.kind, m.view, m.seq = self.kind, self.view, self.seq
        ctypes.memmove(m.digest, bytes(self.digest), 64)
        m.digest_ok = 1
        if self.sig is not None:
            m.has_sig, m.replica = 1, int(self.replica or 0)
            ctypes.memmove(m.sig, bytes(self.sig), 64)
        buf = ctypes.create_string_buffer(bytes(self.operation), max(1, len(self.operation)))
        self._keep = [buf]
        m.operation = ctypes.cast(buf, ctypes.c_void_p)
        m.operation_len = len(self.operation)
        m.timestamp = self.timestamp
        m.client = self.client.encode()
        return m


def uvi_encode(v: int) -> bytes:
    out = (ctypes.c_uint8 * 10)()
    n = load().pbft_uvi_encode(v, out)
    return bytes(out[:n])


def uvi_decode(buf: bytes):
    """(value, header_bytes) | None if more bytes are needed; raises on invalid."""
    v, h = ctypes.c_uint64(), ctypes.c_size_t()
    b = (ctypes.c_uint8 * max(1, len(buf))).from_buffer_copy(buf or b"\0")
    rc = load().pbft_uvi_decode(b, len(buf), ctypes.byref(v), ctypes.byref(h))
    if rc == 1:
        return None
    check(rc)
    return v.value, h.value


def encode_json(m: WireMsg) -> bytes:
    lib, cm = load(), m._to_c()
    n = ctypes.c_size_t()
    lib.pbft_wire_encode_json(ctypes.byref(cm), None, 0, ctypes.byref(n))
    out = ctypes.create_string_buffer(n.value)
    check(lib.pbft_wire_encode_json(ctypes.byref(cm), out, n.value, ctypes.byref(n)))
    return out.raw[: n.value]


def encode_frame(m: WireMsg) -> bytes:
    lib, cm = load(), m._to_c()
    n = ctypes.c_size_t()
    lib.pbft_wire_encode_frame(ctypes.byref(cm), None, 0, ctypes.byref(n))
    out = ctypes.create_string_buffer(n.value)
    check(lib.pbft_wire_encode_frame(ctypes.byref(cm), out, n.value, ctypes.byref(n)))
    return out.raw[: n.value]


def decode_json(js: bytes) -> WireMsg:
    lib = load()
    cm = _Msg()
    arena = ctypes.create_string_buffer(len(js) + 16)
    src = ctypes.create_string_buffer(bytes(js), max(1, len(js)))
    rc = lib.pbft_wire_decode_json(src, len(js), ctypes.byref(cm), arena, len(js) + 16)
    if rc:
        raise PbftError(rc, "not a Message of the reference schema")
    op = ctypes.string_at(cm.operation, cm.operation_len) if cm.operation_len else b""
    return WireMsg(kind=cm.kind, view=cm.view, seq=cm.seq, digest=bytes(cm.digest),
                   replica=cm.replica if cm.has_sig else None, sig=bytes(cm.sig) if cm.has_sig else None,
                   operation=op, timestamp=cm.timestamp, client=cm.client.decode(), digest_ok=bool(cm.digest_ok))


@dataclass
class Votes:
    status: np.ndarray   # per decoded frame (STATUS)
    R: np.ndarray
    S: np.ndarray
    key_idx: np.ndarray
    msg: np.ndarray      # (rows, 85) envelopes
    kind: np.ndarray
    view: np.ndarray
    seq: np.ndarray
    consumed: int        # bytes of whole frames


def decode_votes(stream: bytes, n_replicas: int, max_frames: int | None = None) -> Votes:
    lib = load()
    cap = max(1, len(stream) // 8 + 1) if max_frames is None else max_frames
    st = np.zeros(cap, np.uint8)
    R, S = np.zeros((cap, 32), np.uint8), np.zeros((cap, 32), np.uint8)
    K, M = np.zeros(cap, np.uint16), np.zeros((cap, ENVELOPE), np.uint8)
    kd, vw, sq = np.zeros(cap, np.uint8), np.zeros(cap, np.uint64), np.zeros(cap, np.uint64)
    nf, nr, used = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    buf = np.frombuffer(bytes(stream) or b"\0", np.uint8)
    check(lib.pbft_wire_decode_votes(buf.ctypes.data, len(stream), n_replicas, cap, cap, st.ctypes.data,
                                     R.ctypes.data, S.ctypes.data, K.ctypes.data, M.ctypes.data, kd.ctypes.data,
                                     vw.ctypes.data, sq.ctypes.data, ctypes.byref(nf), ctypes.byref(nr),
                                     ctypes.byref(used)))
    f, r = nf.value, nr.value
    return Votes(st[:f], R[:r], S[:r], K[:r], M[:r], kd[:r], vw[:r], sq[:r], used.value)


def records_pack(R, S, key_idx, msg, msg_stride: int = ENVELOPE) -> np.ndarray:
    n = len(R)
    out = np.zeros((n, RECORD_BYTES), np.uint8)
    R, S = np.ascontiguousarray(R, np.uint8), np.ascontiguousarray(S, np.uint8)
    K, M = np.ascontiguousarray(key_idx, np.uint16), np.ascontiguousarray(msg, np.uint8)
    check(load().pbft_records_pack(R.ctypes.data, S.ctypes.data, K.ctypes.data, M.ctypes.data, msg_stride, n,
                                   out.ctypes.data))
    return out


def encode_votes(kind, view, seq, digests, replica, sigs) -> np.ndarray:
    """N signed votes as one stream of UviBytes/JSON frames (include/pbft_wire.h pbft_wire_encode_votes): what one
    connection carries (uint8 array)."""
    lib = load()
    k = np.ascontiguousarray(kind, np.uint8)
    v, q = np.ascontiguousarray(view, np.uint64), np.ascontiguousarray(seq, np.uint64)
    d, s = np.ascontiguousarray(digests, np.uint8), np.ascontiguousarray(sigs, np.uint8)
    r = np.ascontiguousarray(replica, np.uint32)
    n = ctypes.c_size_t()
    args = (len(k), k.ctypes.data, v.ctypes.data, q.ctypes.data, d.ctypes.data, r.ctypes.data, s.ctypes.data)
    lib.pbft_wire_encode_votes(*args, None, 0, ctypes.byref(n))
    out = np.zeros(max(1, n.value), np.uint8)
    check(lib.pbft_wire_encode_votes(*args, out.ctypes.data, n.value, ctypes.byref(n)))
    return out[: n.value]
