"""Pure-Python restatement of Message::serialize — TEST INFRASTRUCTURE ONLY.

Checker for the serialize half of the host wire codec (wq_serialize_message / wq_serialize_messages
in worldql_server_amd/csrc/wq_codec.cpp). Only tests/ may import it.

It restates, with a bytearray that grows at the front:
* Message::serialize (worldql_server/src/structures/message.rs:120-134): encode, reset the builder,
  MessageT::pack, finish(root, None);
* Message / Record / Entity ::encode (message.rs:28-52, record.rs:18-26, entity.rs:17-25): the
  sender / record uuids as uuid 0.8.2 `to_string()` (lower-case hyphenated), world_name always
  present, records and entities always present (possibly empty vectors), an Entity's position
  always present;
* MessageT::pack and RecordT / EntityT::pack (WorldQLFB_generated.rs:1133-1173, :619-645,
  :838-864) and the create() field order (:1045-1055, :449-457, :668-676);
* the FlatBufferBuilder of crate `flatbuffers` 2.0.0 (Cargo.lock:347-349; not vendored in
  /root/reference, so its published algorithm, src/builder.rs): `align` pads with zeros so the
  next `len` bytes end aligned, strings are NUL + bytes + u32 length under one alignment, vectors
  are written last element first, `push_slot` skips a scalar equal to its default, `write_vtable`
  writes the soffset, then the vtable right below the table, and erases it again when a
  byte-identical vtable was already written in this buffer; `finish` aligns to the largest
  alignment seen and writes the root uoffset. A struct is pushed under its Push::alignment(), whose
  default is align_of::<Output>(): Vec3d (WorldQLFB_generated.rs:254-298) is a repr(transparent)
  [u8; 24] with that default, so positions are pushed with alignment 1 — no padding, min_align
  unchanged — despite the schema's "aligned to 8" comment.

Parity: UNPINNED at the byte level — the reference is Rust, cannot be built here,
and holds no serialized frames. The layout is pinned only by this restatement, by two hand-derived
known-answer frames (tests/test_codec_serialize.py: a Handshake, and a LocalMessage with a position,
one Record and one Entity) and semantically by decoding every frame back
with the verifier restatement in fbs_oracle.py.
"""
from __future__ import annotations

import struct
import uuid as _uuid
from typing import List, Optional

MSG_SLOTS = dict(instruction=4, parameter=6, sender_uuid=8, world_name=10, replication=12, records=14,
                 entities=16, position=18, flex=20)  # WorldQLFB_generated.rs:939-947
REC_SLOTS = dict(uuid=4, position=6, world_name=8, data=10, flex=12)  # :485-489 / :704-708


class _Builder:
    def __init__(self):
        self.buf = bytearray()
        self.min_align = 1
        self.fields: List[tuple] = []
        self.vtables: List[int] = []  # revlocs of the vtables written so far

    def used(self) -> int:
        return len(self.buf)

    def _prepend(self, b: bytes) -> int:
        self.buf[0:0] = b
        return self.used()

    def align(self, n: int, a: int):
        self.min_align = max(self.min_align, a)
        self._prepend(bytes((-(self.used() + n)) % a))

    def u8(self, v: int) -> int:
        return self._prepend(bytes([v]))

    def u32(self, v: int) -> int:
        self.align(4, 4)
        return self._prepend(struct.pack("<I", v))

    def uoffset(self, target: int) -> int:
        self.align(4, 4)
        return self._prepend(struct.pack("<I", self.used() + 4 - target))

    def string(self, raw: bytes) -> int:
        self.align(len(raw) + 1, 4)
        self._prepend(raw + b"\0")
        return self.u32(len(raw))

    def byte_vector(self, raw: bytes) -> int:
        self.align(len(raw), 4)
        self._prepend(raw)
        return self.u32(len(raw))

    def offset_vector(self, targets: List[int]) -> int:
        self.align(4 * len(targets), 4)
        for t in reversed(targets):
            self.uoffset(t)
        return self.u32(len(targets))

    def add(self, slot: int, rev: int):
        self.fields.append((slot, rev))

    def end_table(self, start: int) -> int:
        obj = self.u32(0xF0F0F0F0)
        n = max([s for s, _ in self.fields], default=2) + 2
        vt = bytearray(n)
        struct.pack_into("<HH", vt, 0, n, obj - start)
        for slot, rev in self.fields:
            struct.pack_into("<H", vt, slot, obj - rev)
        self.fields = []
        use = None
        for rev in reversed(self.vtables):
            p = self.used() - rev
            if bytes(self.buf[p:p + n]) == bytes(vt) and struct.unpack_from("<H", self.buf, p)[0] == n:
                use = rev
                break
        if use is None:
            use = self._prepend(bytes(vt))
            self.vtables.append(use)
        struct.pack_into("<i", self.buf, self.used() - obj, use - obj)
        return obj

    def finish(self, root: int) -> bytes:
        self.vtables = []
        self.align(4, self.min_align)
        self.uoffset(root)
        return bytes(self.buf)


def _text(u) -> bytes:
    return str(_uuid.UUID(bytes=bytes(u))).encode()


def _pack_record(b: _Builder, r: dict, entity: bool) -> int:
    uu = b.string(_text(r["uuid"]))
    world = b.string(r["world_name"].encode())
    data = b.string(r["data"].encode()) if r.get("data") is not None else None
    flex = b.byte_vector(bytes(r["flex"])) if r.get("flex") is not None else None
    start = b.used()
    if flex is not None:
        b.add(REC_SLOTS["flex"], b.uoffset(flex))
    if data is not None:
        b.add(REC_SLOTS["data"], b.uoffset(data))
    b.add(REC_SLOTS["world_name"], b.uoffset(world))
    pos = r.get("position")
    if entity or pos is not None:
        b.add(REC_SLOTS["position"], b._prepend(struct.pack("<3d", *(pos or (0.0, 0.0, 0.0)))))
    b.add(REC_SLOTS["uuid"], b.uoffset(uu))
    return b.end_table(start)


def serialize(m: dict) -> bytes:
    """m: instruction (wire code), replication, sender_uuid (16 bytes), world_name (str), and optional
    parameter (str), position (x, y, z), flex (bytes), records / entities (lists of dicts with uuid,
    world_name, and optional position / data / flex)."""
    b = _Builder()
    param: Optional[int] = b.string(m["parameter"].encode()) if m.get("parameter") is not None else None
    sender = b.string(_text(m["sender_uuid"]))
    world = b.string(m["world_name"].encode())
    recs = b.offset_vector([_pack_record(b, r, False) for r in m.get("records", [])])
    ents = b.offset_vector([_pack_record(b, e, True) for e in m.get("entities", [])])
    flex = b.byte_vector(bytes(m["flex"])) if m.get("flex") is not None else None
    start = b.used()
    if flex is not None:
        b.add(MSG_SLOTS["flex"], b.uoffset(flex))
    if m.get("position") is not None:
        b.add(MSG_SLOTS["position"], b._prepend(struct.pack("<3d", *m["position"])))
    b.add(MSG_SLOTS["entities"], b.uoffset(ents))
    b.add(MSG_SLOTS["records"], b.uoffset(recs))
    b.add(MSG_SLOTS["world_name"], b.uoffset(world))
    b.add(MSG_SLOTS["sender_uuid"], b.uoffset(sender))
    if param is not None:
        b.add(MSG_SLOTS["parameter"], b.uoffset(param))
    if m.get("replication", 0) != 0:  # ExceptSelf is the default
        b.add(MSG_SLOTS["replication"], b.u8(m["replication"]))
    if m.get("instruction", 0) != 0:  # Heartbeat is the default
        b.add(MSG_SLOTS["instruction"], b.u8(m["instruction"]))
    return b.finish(b.end_table(start))
