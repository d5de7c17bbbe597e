"""Serialize half of the host wire codec: wq_serialize_message(s) of
libwq_router.so against the Python restatement oracle/fbs_serialize.py (byte for byte), a
hand-derived known-answer frame, and the decoders (C++ wq_decode_messages and oracle/fbs_oracle.py)
reading every field back. CPU only.

Parity: byte layout UNPINNED against the reference itself (Rust flatbuffers 2.0.0 builder; no
serialized frames exist in /root/reference) — see oracle/fbs_serialize.py.
"""
import os
import random
import struct
import sys
import uuid

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import fbs_oracle, fbs_serialize  # noqa: E402

codec = pytest.importorskip("worldql_server_amd.codec")


def _handshake_kat() -> bytes:
    """Message { instruction: Handshake, ..Default } as outgoing.rs:110-116 sends it, laid out by hand
    following the builder (revloc = bytes used from the end; the frame is 108 bytes):
      sender "0000…" : pad 3, NUL, 36 chars, len 36            -> revloc 44
      world ""       : pad 3, NUL, len 0                        -> revloc 52
      records []     : len 0 -> 56;  entities [] : len 0 -> 60 (table start)
      slots in create() order: entities (64), records (68), world (72), sender (76), instruction u8 (77)
      soffset        : pad 3, i32 -> revloc 84 (object size 84 - 60 = 24)
      vtable         : 18 bytes (highest slot 16) -> revloc 102, soffset = 102 - 84 = 18
      finish         : pad 2 (104), root uoffset 108 - 84 = 24
    """
    vt = struct.pack("<9H", 18, 24, 84 - 77, 0, 84 - 76, 84 - 72, 0, 84 - 68, 84 - 64)
    table = struct.pack("<i", 18) + b"\0\0\0" + b"\x01" + struct.pack("<4I", 64 - 32, 56 - 36, 52 - 40, 48 - 44)
    tail = struct.pack("<I", 0) * 2 + struct.pack("<I", 0) + b"\0" * 4 + struct.pack("<I", 36) + \
        str(uuid.UUID(int=0)).encode() + b"\0" * 4
    return struct.pack("<I", 24) + b"\0\0" + vt + table + tail


def _local_message_kat() -> bytes:
    """LocalMessage { sender 0…0, world "w", position (1, 2, 3), records [Record { uuid 0…0, world "w",
    data "d" }], entities [Entity { uuid 0…0, world "w", position (4, 5, 6) }] }, laid out by hand in
    MessageT::pack order (WorldQLFB_generated.rs:1133-1173; RecordT/EntityT::pack :619-645, :838-864)
    — 328 bytes. Vec3d (:254-298) is `#[repr(transparent)] struct Vec3d([u8; 24])` and its Push impl
    keeps the trait's default alignment, align_of::<Vec3d>() = 1 (flatbuffers 2.0.0 src/push.rs), so a
    position is pushed with NO padding and does not raise min_align: the message position lands at
    byte 48 and the entity's at byte 100 (not 8-aligned), although the schema comment says "aligned
    to 8". revloc = bytes used from the end after each step:
      sender : pad 3, NUL, 36, len                                     -> 44
      world  : pad 2, "w" NUL, len                                     -> 52
      record : uuid str -> 96, world str -> 104, data str -> 112 (table start);
               data @116 (4), world @120 (16), uuid @124 (28), soffset -> 128 (size 16);
               vtable 12 bytes (slots 4, 6 = 0, 8, 10) -> 140, soffset 12
      records: uoffset 16 -> 144, len 1 -> 148
      entity : uuid str -> 192, world str -> 200 (table start);
               world @204 (4), position 24 bytes @228 (no pad), uuid @232 (40), soffset -> 236 (size 36);
               vtable 10 bytes (slots 4, 6, 8) -> 246, soffset 10
      entities: pad 2 -> 248, uoffset 16 -> 252, len 1 -> 256 (message table start)
      message: position @280, entities @284 (28), records @288 (140), world @292 (240),
               sender @296 (252), replication 0 = default (omitted), instruction 7 @297,
               pad 3, soffset -> 304 (size 48); vtable 20 bytes (slot 18) -> 324, soffset 20
      finish : min_align 4, no pad; root uoffset 328 - 304 = 24
    """
    zero = str(uuid.UUID(int=0)).encode()

    def s(raw):  # len, bytes, NUL, zero pad to 4
        b = struct.pack("<I", len(raw)) + raw + b"\0"
        return b + b"\0" * (-len(b) % 4)

    msg_vt = struct.pack("<10H", 20, 48, 7, 0, 8, 12, 0, 16, 20, 24)
    msg_table = struct.pack("<i", 20) + b"\0\0\0\x07" + struct.pack("<4I", 252, 240, 140, 28) + \
        struct.pack("<3d", 1.0, 2.0, 3.0)
    ents = struct.pack("<2I", 1, 16) + b"\0\0"
    ent_vt = struct.pack("<5H", 10, 36, 4, 8, 32)
    ent_table = struct.pack("<iI", 10, 40) + struct.pack("<3d", 4.0, 5.0, 6.0) + struct.pack("<I", 4)
    recs = struct.pack("<2I", 1, 16)
    rec_vt = struct.pack("<6H", 12, 16, 4, 0, 8, 12)
    rec_table = struct.pack("<i3I", 12, 28, 16, 4)
    out = struct.pack("<I", 24) + msg_vt + msg_table + ents + ent_vt + ent_table + s(b"w") + s(zero) + \
        recs + rec_vt + rec_table + s(b"d") + s(b"w") + s(zero) + s(b"w") + s(zero)
    assert struct.unpack_from("<3d", out, 48) == (1.0, 2.0, 3.0) and struct.unpack_from("<3d", out, 100) == (4.0, 5.0, 6.0)
    return out


def test_local_message_known_answer():
    want = _local_message_kat()
    assert len(want) == 328
    z = bytes(16)
    m = dict(instruction=7, sender_uuid=z, world_name="w", position=(1.0, 2.0, 3.0),
             records=[dict(uuid=z, world_name="w", data="d")],
             entities=[dict(uuid=z, world_name="w", position=(4.0, 5.0, 6.0))])
    assert fbs_serialize.serialize(m) == want
    assert codec.serialize_message(m) == want
    assert read_back(want) == _normal(m)
    d = fbs_oracle.decode(want)
    assert d["status"] == 0 and d["instruction"] == 7 and d["world"] == b"w"
    assert d["n_records"] == 1 and d["n_entities"] == 1


def test_handshake_known_answer():
    want = _handshake_kat()
    assert len(want) == 108
    m = dict(instruction=1, sender_uuid=bytes(16), world_name="")
    assert fbs_serialize.serialize(m) == want
    assert codec.serialize_message(m) == want
    d = fbs_oracle.decode(want)
    assert d["status"] == 0 and d["instruction"] == 1 and d["world"] == b"" and d["n_records"] == 0


# ---- a generic reader: every field of a frame back out ------------------------------------------

def _tab(b, pos):
    vt = pos - struct.unpack_from("<i", b, pos)[0]
    vl = struct.unpack_from("<H", b, vt)[0]

    def fld(slot):
        if slot >= vl:
            return None
        o = struct.unpack_from("<H", b, vt + slot)[0]
        return pos + o if o else None
    return fld


def _follow(b, p):
    return p + struct.unpack_from("<I", b, p)[0]


def _vec(b, p):
    n = struct.unpack_from("<I", b, p)[0]
    return b[p + 4:p + 4 + n]


def _record(b, pos, entity):
    f = _tab(b, pos)
    S = fbs_serialize.REC_SLOTS
    r = dict(uuid=uuid.UUID(_vec(b, _follow(b, f(S["uuid"]))).decode()).bytes,
             world_name=_vec(b, _follow(b, f(S["world_name"]))).decode())
    if f(S["position"]) is not None:
        r["position"] = struct.unpack_from("<3d", b, f(S["position"]))
    if f(S["data"]) is not None:
        r["data"] = _vec(b, _follow(b, f(S["data"]))).decode()
    if f(S["flex"]) is not None:
        r["flex"] = _vec(b, _follow(b, f(S["flex"])))
    return r


def read_back(b: bytes) -> dict:
    f = _tab(b, _follow(b, 0))
    S = fbs_serialize.MSG_SLOTS
    m = dict(instruction=b[f(S["instruction"])] if f(S["instruction"]) else 0,
             replication=b[f(S["replication"])] if f(S["replication"]) else 0,
             sender_uuid=uuid.UUID(_vec(b, _follow(b, f(S["sender_uuid"]))).decode()).bytes,
             world_name=_vec(b, _follow(b, f(S["world_name"]))).decode())
    if f(S["parameter"]) is not None:
        m["parameter"] = _vec(b, _follow(b, f(S["parameter"]))).decode()
    if f(S["position"]) is not None:
        m["position"] = struct.unpack_from("<3d", b, f(S["position"]))
    if f(S["flex"]) is not None:
        m["flex"] = _vec(b, _follow(b, f(S["flex"])))
    for name, ent in (("records", False), ("entities", True)):
        p = _follow(b, f(S[name]))  # always present (Some(vec![]) when empty)
        n = struct.unpack_from("<I", b, p)[0]
        m[name] = [_record(b, _follow(b, p + 4 + 4 * i), ent) for i in range(n)]
    return m


WORDS = ["world", "w42", "chat/server_1", "ünïcode €", "", "x" * 70]


def _rand_record(r, entity):
    d = dict(uuid=r.getrandbits(128).to_bytes(16, "big"), world_name=r.choice(WORDS))
    if entity or r.random() < 0.5:
        d["position"] = (r.uniform(-1e5, 1e5), r.choice([0.0, -0.0, 1.5]), r.uniform(-1, 1))
    if r.random() < 0.5:
        d["data"] = r.choice(WORDS) * r.randrange(0, 3)
    if r.random() < 0.4:
        d["flex"] = bytes(r.getrandbits(8) for _ in range(r.randrange(0, 13)))
    return d


def rand_message(r):
    m = dict(instruction=r.choice([0, 1, 4, 5, 6, 7, 12, 255]), replication=r.choice([0, 1, 2]),
             sender_uuid=r.getrandbits(128).to_bytes(16, "big"), world_name=r.choice(WORDS))
    if r.random() < 0.6:
        m["position"] = (r.uniform(-1e4, 1e4), r.uniform(-1e4, 1e4), r.uniform(-1e4, 1e4))
    if r.random() < 0.3:
        m["parameter"] = r.choice(WORDS)
    if r.random() < 0.3:
        m["flex"] = bytes(r.getrandbits(8) for _ in range(r.randrange(0, 40)))
    m["records"] = [_rand_record(r, False) for _ in range(r.choice([0, 0, 1, 3]))]
    m["entities"] = [_rand_record(r, True) for _ in range(r.choice([0, 0, 1, 2]))]
    return m


def _normal(m):
    """The fields as Message::encode writes them (defaults filled in)."""
    out = dict(instruction=m.get("instruction", 255), replication=m.get("replication", 0),
               sender_uuid=bytes(m["sender_uuid"]), world_name=m["world_name"])
    for k in ("parameter", "position", "flex"):
        if m.get(k) is not None:
            out[k] = tuple(m[k]) if k == "position" else (bytes(m[k]) if k == "flex" else m[k])
    for name, ent in (("records", False), ("entities", True)):
        rs = []
        for x in m.get(name, []):
            y = dict(uuid=x["uuid"], world_name=x["world_name"])
            if ent or x.get("position") is not None:
                y["position"] = tuple(x.get("position") or (0.0, 0.0, 0.0))
            if x.get("data") is not None:
                y["data"] = x["data"]
            if x.get("flex") is not None:
                y["flex"] = bytes(x["flex"])
            rs.append(y)
        out[name] = rs
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_messages_match_restatement_and_read_back(seed):
    r = random.Random(seed)
    for _ in range(300):
        m = rand_message(r)
        got = codec.serialize_message(m)
        assert got == fbs_serialize.serialize(m)
        assert len(got) % 4 == 0
        assert read_back(got) == _normal(m)
        d = fbs_oracle.decode(got)
        assert d["status"] == 0, m
        assert d["world"] == m["world_name"].encode() and d["sender_uuid"] == m["sender_uuid"]
        assert d["n_records"] == len(m["records"]) and d["n_entities"] == len(m["entities"])


def test_batch_equals_single_frames_and_decodes():
    r = random.Random(9)
    msgs = [rand_message(r) for _ in range(5000)]
    data, offsets = codec.serialize_messages(msgs, n_threads=1)
    data8, offsets8 = codec.serialize_messages(msgs, n_threads=8)
    assert np.array_equal(offsets, offsets8) and data.tobytes() == data8.tobytes()
    for i in range(0, len(msgs), 97):
        assert data[offsets[i]:offsets[i + 1]].tobytes() == codec.serialize_message(msgs[i])
    recs = codec.decode_packed(data, offsets)
    assert (recs["status"] == codec.DEC_OK).all()
    ins = np.array([m["instruction"] for m in msgs])
    np.testing.assert_array_equal(recs["instruction"], np.where(ins <= 12, ins, 255))
    np.testing.assert_array_equal(recs["replication"], [m["replication"] for m in msgs])
    np.testing.assert_array_equal(recs["has_position"], [m.get("position") is not None for m in msgs])
    np.testing.assert_array_equal(recs["n_records"], [len(m["records"]) for m in msgs])
    np.testing.assert_array_equal(recs["n_entities"], [len(m["entities"]) for m in msgs])
    for i in range(0, len(msgs), 53):
        f = data[offsets[i]:offsets[i + 1]].tobytes()
        w0, wl = int(recs[i]["world_off"]), int(recs[i]["world_len"])
        assert f[w0:w0 + wl].decode() == msgs[i]["world_name"]
        assert bytes(recs[i]["sender_uuid"]) == msgs[i]["sender_uuid"]


def test_vtables_shared_within_a_frame():
    """Records of one shape share one vtable: every record table's soffset lands on one place."""
    u = bytes(range(16))
    recs = [dict(uuid=u, world_name="w", data="d") for _ in range(6)]
    b = codec.serialize_message(dict(instruction=7, sender_uuid=u, world_name="w", records=recs))
    f = _tab(b, _follow(b, 0))
    p = _follow(b, f(fbs_serialize.MSG_SLOTS["records"]))
    vts = set()
    for i in range(6):
        t = _follow(b, p + 4 + 4 * i)
        vts.add(t - struct.unpack_from("<i", b, t)[0])
    assert len(vts) == 1
    one = codec.serialize_message(dict(instruction=7, sender_uuid=u, world_name="w", records=recs[:1]))
    # five more records cost their tables and strings, not five more vtables
    # uuid string 44 + "w" 8 + "d" 8 + table (soffset + 3 uoffsets) 16 + its vector entry 4; a vtable
    # of its own (highest slot 10) would add 12
    assert len(b) - len(one) == 5 * 80


def test_empty_batch_and_errors():
    data, offsets = codec.serialize_messages([])
    assert len(data) == 0 and offsets.tolist() == [0]
    with pytest.raises(ValueError, match="UTF-8"):
        codec.serialize_message(dict(instruction=7, sender_uuid=bytes(16), world_name=b"\xff\xfe"))
    with pytest.raises(ValueError, match="UTF-8"):
        codec.serialize_messages([dict(instruction=7, sender_uuid=bytes(16), world_name="ok",
                                       records=[dict(uuid=bytes(16), world_name="w", data=b"\xc0\x80")])])


def test_routed_local_message_round_trip():
    """A LocalMessage as the tick forwards it (local_message.rs: the received Message itself is
    serialized once for every recipient): decode -> serialize -> decode keeps every routed field."""
    from fbs_builder import message
    u = str(uuid.UUID(int=12345))
    src = message(instruction=7, sender_uuid=u, world_name="chat/server_1", position=(1.5, -2.25, 1e9),
                  replication=2, parameter="hello")
    ev = codec.decode_batch([src])[0]
    frame = codec.serialize_message(dict(instruction=int(ev["instruction"]), replication=int(ev["replication"]),
                                         sender_uuid=bytes(ev["sender_uuid"]), world_name="chat/server_1",
                                         position=tuple(ev["position"]), parameter="hello"))
    back = codec.decode_batch([frame])[0]
    for k in ("status", "instruction", "replication", "has_position", "has_parameter"):
        assert back[k] == ev[k], k
    assert bytes(back["sender_uuid"]) == bytes(ev["sender_uuid"])
    assert np.array_equal(back["position"], ev["position"])
