"""Python binding of the host wire codec (include/wq_codec.h).

`decode_batch` runs the C++ batch decoder of libwq_router.so (wq_codec.cpp) over a list of
received frames: FlatBuffers verification and Message decode as in
worldql_server/src/structures/message.rs:136-142 / :60-114, one structured record per frame.
`decode_messages` turns those records into the `processing.Message` events the tick loop takes,
dropping frames that fail to decode exactly as the ZeroMQ ingress does
(transport/zeromq/incoming.rs:39-45). `sanitize_world_name` is the C restatement of
utils/world_names.rs:54-87. `serialize_message` / `serialize_messages` are the egress half: the C++
restatement of Message::serialize (message.rs:120-134, a flatbuffers 2.0.0 builder) for one frame
or a whole tick's routed messages. Host code only: no GPU is needed.
"""
from __future__ import annotations

import ctypes
import uuid as _uuid
from typing import List, Optional, Sequence

import numpy as np

from .router import load_library
from .subscriptions import Vector3

DEC_OK, DEC_INVALID_FLATBUFFER, DEC_MISSING_FIELD, DEC_BAD_UUID = 0, 1, 2, 3
INSTRUCTION_NAMES = ["Heartbeat", "Handshake", "PeerConnect", "PeerDisconnect", "AreaSubscribe",
                     "AreaUnsubscribe", "GlobalMessage", "LocalMessage", "RecordCreate", "RecordRead",
                     "RecordUpdate", "RecordDelete", "RecordReply"]  # WorldQLFB_generated.rs:56-68
SANITIZE_ERRORS = {1: "IsGlobalWorld", 2: "ZeroLength", 3: "InvalidStart", 4: "InvalidChars", 5: "TooLong"}

# struct wq_decoded_msg (include/wq_codec.h), 72 bytes
DECODED_DTYPE = np.dtype([
    ("status", np.int32), ("instruction", np.uint8), ("replication", np.uint8),
    ("has_position", np.uint8), ("has_parameter", np.uint8), ("sender_uuid", np.uint8, (16,)),
    ("position", np.float64, (3,)), ("world_off", np.uint32), ("world_len", np.uint32),
    ("param_off", np.uint32), ("param_len", np.uint32), ("n_records", np.uint32), ("n_entities", np.uint32),
])
assert DECODED_DTYPE.itemsize == 72

SER_ERRORS = {-1: "invalid arguments", -2: "output too small", -3: "string field is not UTF-8",
              -4: "frame exceeds the builder's 2 GiB limit"}


class WqRecordIn(ctypes.Structure):
    """struct wq_record_in (include/wq_codec.h): a Record or an Entity."""
    _fields_ = [("uuid", ctypes.c_uint8 * 16), ("has_position", ctypes.c_uint8), ("has_data", ctypes.c_uint8),
                ("has_flex", ctypes.c_uint8), ("pad_", ctypes.c_uint8 * 5), ("position", ctypes.c_double * 3),
                ("world_name", ctypes.c_char_p), ("world_len", ctypes.c_uint64),
                ("data", ctypes.c_char_p), ("data_len", ctypes.c_uint64),
                ("flex", ctypes.c_char_p), ("flex_len", ctypes.c_uint64)]


class WqMessageIn(ctypes.Structure):
    """struct wq_message_in (include/wq_codec.h)."""
    _fields_ = [("instruction", ctypes.c_uint8), ("replication", ctypes.c_uint8), ("has_position", ctypes.c_uint8),
                ("has_parameter", ctypes.c_uint8), ("has_flex", ctypes.c_uint8), ("pad_", ctypes.c_uint8 * 3),
                ("sender_uuid", ctypes.c_uint8 * 16), ("position", ctypes.c_double * 3),
                ("parameter", ctypes.c_char_p), ("parameter_len", ctypes.c_uint64),
                ("world_name", ctypes.c_char_p), ("world_len", ctypes.c_uint64),
                ("flex", ctypes.c_char_p), ("flex_len", ctypes.c_uint64),
                ("records", ctypes.POINTER(WqRecordIn)), ("n_records", ctypes.c_uint64),
                ("entities", ctypes.POINTER(WqRecordIn)), ("n_entities", ctypes.c_uint64)]


assert ctypes.sizeof(WqRecordIn) == 96 and ctypes.sizeof(WqMessageIn) == 128

_sig_done = False


def _lib():
    global _sig_done
    lib = load_library()
    if not _sig_done:
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.wq_decode_messages.argtypes = [vp, vp, sz, vp, ctypes.c_int]
        lib.wq_decode_messages.restype = ctypes.c_int
        lib.wq_sanitize_world_name.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        lib.wq_sanitize_world_name.restype = ctypes.c_int
        lib.wq_serialize_message.argtypes = [ctypes.POINTER(WqMessageIn), vp, sz, ctypes.POINTER(sz)]
        lib.wq_serialize_message.restype = ctypes.c_int
        lib.wq_serialize_messages.argtypes = [vp, sz, vp, sz, vp, ctypes.c_int]
        lib.wq_serialize_messages.restype = ctypes.c_int
        lib.wq_serialize_bound.argtypes = [vp, sz]
        lib.wq_serialize_bound.restype = sz
        _sig_done = True
    return lib


def pack_frames(frames: Sequence[bytes]):
    """Concatenate frames into one byte array + n+1 offsets (the decoder's input layout)."""
    lens = np.fromiter((len(f) for f in frames), dtype=np.uint64, count=len(frames))
    offsets = np.zeros(len(frames) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    data = np.frombuffer(b"".join(frames), dtype=np.uint8) if frames else np.zeros(0, np.uint8)
    return data, offsets


def decode_packed(data: np.ndarray, offsets: np.ndarray, n_threads: int = 0, out=None) -> np.ndarray:
    """`out`: a reusable DECODED_DTYPE array of at least n records (a server keeps one per tick)."""
    n = len(offsets) - 1
    if out is None:
        out = np.zeros(max(n, 0), dtype=DECODED_DTYPE)
    elif out.dtype != DECODED_DTYPE or len(out) < n or not out.flags.c_contiguous:
        raise ValueError("out: a contiguous DECODED_DTYPE array of >= n records")
    if n <= 0:
        return out
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    buf = data if len(data) else np.zeros(1, np.uint8)
    rc = _lib().wq_decode_messages(buf.ctypes.data, offsets.ctypes.data, n, out.ctypes.data, int(n_threads))
    if rc != 0:
        raise ValueError(f"wq_decode_messages: invalid arguments ({rc})")
    return out[:n]


def decode_batch(frames: Sequence[bytes], n_threads: int = 0) -> np.ndarray:
    """One DECODED_DTYPE record per frame (byte ranges are relative to each frame)."""
    data, offsets = pack_frames(frames)
    return decode_packed(data, offsets, n_threads)


def decode_messages(frames: Sequence[bytes], n_threads: int = 0):
    """`processing.Message` per frame, or None where Message::deserialize fails (the frame the
    ingress drops). Instruction codes outside 0..12 become "Unknown"."""
    from .processing import Message
    recs = decode_batch(frames, n_threads)
    out: List[Optional[Message]] = []
    for f, r in zip(frames, recs):
        if r["status"] != DEC_OK:
            out.append(None)
            continue
        ins = int(r["instruction"])
        w0, wl = int(r["world_off"]), int(r["world_len"])
        pos = Vector3(*map(float, r["position"])) if r["has_position"] else None
        out.append(Message(instruction=INSTRUCTION_NAMES[ins] if ins < len(INSTRUCTION_NAMES) else "Unknown",
                           sender_uuid=_uuid.UUID(bytes=bytes(r["sender_uuid"])),
                           world_name=f[w0:w0 + wl].decode("utf-8"), position=pos,
                           replication=int(r["replication"])))
    return out


class SanitizeCError(ValueError):
    def __init__(self, kind: str):
        super().__init__(kind)
        self.kind = kind


def sanitize_world_name(name: str) -> str:
    """C restatement of world_names.rs:54-87 (raises SanitizeCError with the variant name)."""
    raw = name.encode("utf-8")
    out = ctypes.create_string_buffer(64)
    n = ctypes.c_size_t(0)
    rc = _lib().wq_sanitize_world_name(raw, len(raw), out, 64, ctypes.byref(n))
    if rc != 0:
        raise SanitizeCError(SANITIZE_ERRORS.get(rc, f"error {rc}"))
    return out.raw[:n.value].decode("ascii")


# ---- serialize (egress) ----------------------------------------------------------------------

def _uuid16(u) -> bytes:
    if isinstance(u, _uuid.UUID):
        return u.bytes
    b = bytes(u)
    if len(b) != 16:
        raise ValueError("uuid: 16 bytes or uuid.UUID")
    return b


def _utf8(s) -> bytes:
    return s if isinstance(s, (bytes, bytearray)) else s.encode("utf-8")


def _fill_record(dst: WqRecordIn, r: dict, keep: list):
    dst.uuid[:] = _uuid16(r["uuid"])
    w = _utf8(r.get("world_name", ""))
    keep.append(w)
    dst.world_name, dst.world_len = w, len(w)
    pos = r.get("position")
    dst.has_position = pos is not None
    if pos is not None:
        dst.position[:] = [float(v) for v in pos]
    if r.get("data") is not None:
        d = _utf8(r["data"])
        keep.append(d)
        dst.has_data, dst.data, dst.data_len = 1, d, len(d)
    if r.get("flex") is not None:
        f = bytes(r["flex"])
        keep.append(f)
        dst.has_flex, dst.flex, dst.flex_len = 1, f, len(f)


def _message_in(m: dict, keep: list) -> WqMessageIn:
    """m: instruction (wire code, default 255 = Unknown as Message::default), replication, sender_uuid,
    world_name, and optional parameter / position / flex / records / entities (lists of dicts)."""
    o = WqMessageIn()
    o.instruction = int(m.get("instruction", 255))
    o.replication = int(m.get("replication", 0))
    o.sender_uuid[:] = _uuid16(m.get("sender_uuid", bytes(16)))
    w = _utf8(m.get("world_name", ""))
    keep.append(w)
    o.world_name, o.world_len = w, len(w)
    if m.get("parameter") is not None:
        p = _utf8(m["parameter"])
        keep.append(p)
        o.has_parameter, o.parameter, o.parameter_len = 1, p, len(p)
    if m.get("position") is not None:
        o.has_position = 1
        o.position[:] = [float(v) for v in m["position"]]
    if m.get("flex") is not None:
        f = bytes(m["flex"])
        keep.append(f)
        o.has_flex, o.flex, o.flex_len = 1, f, len(f)
    for name in ("records", "entities"):
        rs = m.get(name) or []
        arr = (WqRecordIn * max(len(rs), 1))()
        for i, r in enumerate(rs):
            _fill_record(arr[i], r, keep)
        keep.append(arr)
        setattr(o, name, ctypes.cast(arr, ctypes.POINTER(WqRecordIn)))
        setattr(o, "n_" + name, len(rs))
    return o


def _ser_check(rc: int, what: str):
    if rc != 0:
        raise ValueError(f"{what}: {SER_ERRORS.get(rc, rc)}")


def serialize_message(m: dict) -> bytes:
    """Message::serialize (message.rs:120-134) of one message (see `_message_in` for the dict)."""
    keep: list = []
    o = _message_in(m, keep)
    n = ctypes.c_size_t(0)
    lib = _lib()
    rc = lib.wq_serialize_message(ctypes.byref(o), None, 0, ctypes.byref(n))
    if rc == -2:
        out = ctypes.create_string_buffer(max(n.value, 1))
        rc = lib.wq_serialize_message(ctypes.byref(o), out, n.value, ctypes.byref(n))
        _ser_check(rc, "wq_serialize_message")
        return out.raw[:n.value]
    _ser_check(rc, "wq_serialize_message")
    return b""


def serialize_messages(msgs: Sequence[dict], n_threads: int = 0):
    """Frames of a whole batch: (data uint8 array, offsets uint64 array of n + 1) — the decoder's
    input layout, so `decode_packed(*serialize_messages(ms))` round-trips."""
    keep: list = []
    arr = (WqMessageIn * max(len(msgs), 1))()
    for i, m in enumerate(msgs):
        arr[i] = _message_in(m, keep)
    offsets = np.zeros(len(msgs) + 1, dtype=np.uint64)
    lib = _lib()
    cap = lib.wq_serialize_bound(ctypes.addressof(arr), len(msgs))  # packed in place, one pass
    data = np.empty(max(cap, 1), dtype=np.uint8)
    rc = lib.wq_serialize_messages(ctypes.addressof(arr), len(msgs), data.ctypes.data, cap, offsets.ctypes.data,
                                   int(n_threads))
    _ser_check(rc, "wq_serialize_messages")
    return data[:int(offsets[-1])], offsets
