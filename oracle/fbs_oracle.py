"""Pure-Python restatement of Message::deserialize — TEST INFRASTRUCTURE ONLY.

Checker for the host wire codec (worldql_server_amd/csrc/wq_codec.cpp). Only
tests/ may import it. It restates, in plain Python loops:

* the FlatBuffers 2.0.0 Rust verifier (crate `flatbuffers` 2.0.0, Cargo.lock:347-349; not vendored
  in /root/reference, so its published algorithm, src/verifier.rs) as `root_as_message` runs it
  (worldql_server/src/flatbuffers/WorldQLFB_generated.rs:1192-1194) over the Message table
  (:986-1004), Record (:515-527) and Entity (:734-746): uoffsets / soffsets aligned relative to the
  buffer start and in range, vtable length even and in range, strings UTF-8 with a NUL after
  them, vectors in range, Vec3d (alignment 1, 24 bytes) in range;
* MessageT -> Message (structures/message.rs:60-114): world_name, sender_uuid required; every
  Record (record.rs:30-50) and Entity (entity.rs:29-48) decoded; Instruction codes outside 0..12
  -> Unknown (instruction.rs:57-76), Replication codes outside 0..2 -> ExceptSelf
  (replication.rs:34-43);
* uuid 0.8.2's `Uuid::parse_str` (Cargo.lock:1674-1676; not vendored): urn prefix, simple or
  hyphenated forms, hex digits of either case.

Parity: the reference is Rust and cannot be built or run here and holds no
FlatBuffers frames or uuid vectors of its own, so the codec's results on malformed frames are
"parity unpinned" beyond this restatement; valid frames are pinned by construction (the
independent builder in tests/fbs_builder.py writes the fields the decoder must return).
"""
from __future__ import annotations

import struct

OK, INVALID_FLATBUFFER, MISSING_FIELD, BAD_UUID = 0, 1, 2, 3
MAX_TABLES = 1_000_000
MAX_DEPTH = 64
MAX_APPARENT = 1 << 31


class _Invalid(Exception):
    pass


class _V:
    def __init__(self, buf: bytes):
        self.b = buf
        self.apparent = 0
        self.tables = 0
        self.depth = 0

    def aligned(self, pos, a):
        if pos % a:
            raise _Invalid("unaligned")

    def rng(self, pos, size):
        if pos + size > len(self.b):
            raise _Invalid("range")
        self.apparent += size
        if self.apparent > MAX_APPARENT:
            raise _Invalid("apparent size")

    def u32(self, pos):
        self.aligned(pos, 4)
        self.rng(pos, 4)
        return struct.unpack_from("<I", self.b, pos)[0]

    def u16(self, pos):
        self.aligned(pos, 2)
        self.rng(pos, 2)
        return struct.unpack_from("<H", self.b, pos)[0]

    def follow(self, pos):
        return pos + self.u32(pos)

    def vec(self, pos, elem):
        n = self.u32(pos)
        start = pos + 4
        self.aligned(start, elem)
        self.rng(start, n * elem)
        return start, n

    def string(self, pos):
        self.aligned(pos, 4)
        start, n = self.vec(pos, 1)
        raw = self.b[start:start + n]
        try:
            raw.decode("utf-8")  # Python's strict decoder = Rust's from_utf8 acceptance
        except UnicodeDecodeError:
            raise _Invalid("utf8")
        if start + n >= len(self.b) or self.b[start + n] != 0:
            raise _Invalid("missing NUL")
        return raw

    def table(self, pos):
        self.tables += 1
        if self.tables > MAX_TABLES:
            raise _Invalid("too many tables")
        so = struct.unpack("<i", struct.pack("<I", self.u32(pos)))[0]
        vt = pos - so
        if vt < 0 or vt >= len(self.b):
            raise _Invalid("soffset")
        vl = self.u16(vt)
        self.aligned(vt + vl, 2)
        self.rng(vt, vl)
        self.depth += 1
        if self.depth > MAX_DEPTH:
            raise _Invalid("depth")
        return pos, vt, vl

    def field(self, t, voff):
        pos, vt, vl = t
        if voff < vl:
            fo = self.u16(vt + voff)
            if fo:
                return pos + fo
        return None


def parse_uuid(s: bytes):
    """uuid 0.8.2 Uuid::parse_str -> 16 bytes, or None."""
    if len(s) == 45 and s.startswith(b"urn:uuid:"):
        s = s[9:]
    elif len(s) not in (32, 36):
        return None
    ends = [8, 12, 16, 20, 32]
    out = bytearray(16)
    digit = group = acc = 0
    hexd = b"0123456789abcdefABCDEF"
    for c in s:
        if digit >= 32 and group != 4:
            return None
        if digit % 2 == 0:
            if c in hexd:
                acc = int(chr(c), 16)
            elif c == ord("-"):
                if group > 4 or ends[group] != digit:
                    return None
                group += 1
                digit -= 1
            else:
                return None
        else:
            if c not in hexd:
                return None
            acc = acc * 16 + int(chr(c), 16)
            out[digit // 2] = acc
        digit += 1
    return bytes(out) if digit == 32 else None


def _record_like(v: _V, pos: int, entity: bool):
    """Verify a Record / Entity table; return its decode status (raises _Invalid)."""
    t = v.table(pos)
    f = v.field(t, 4)
    uuid = v.string(v.follow(f)) if f is not None else None
    f = v.field(t, 6)
    has_pos = f is not None
    if has_pos:
        v.rng(f, 24)
    f = v.field(t, 8)
    world = v.string(v.follow(f)) if f is not None else None
    f = v.field(t, 10)
    if f is not None:
        v.string(v.follow(f))
    f = v.field(t, 12)
    if f is not None:
        p = v.follow(f)
        v.aligned(p, 4)
        v.vec(p, 1)
    v.depth -= 1
    if uuid is None or (entity and not has_pos) or world is None:
        return MISSING_FIELD
    return OK if parse_uuid(uuid) is not None else BAD_UUID


def _tables(v: _V, t, voff, entity):
    f = v.field(t, voff)
    if f is None:
        return 0, OK
    p = v.follow(f)
    v.aligned(p, 4)
    start, n = v.vec(p, 4)
    dec = OK
    for i in range(n):
        s = _record_like(v, v.follow(start + 4 * i), entity)
        if dec == OK:
            dec = s
    return n, dec


def decode(buf: bytes) -> dict:
    """Message::deserialize of one frame -> dict of the fields wq_decoded_msg carries."""
    v = _V(bytes(buf))
    out = {"status": OK}
    try:
        t = v.table(v.follow(0))
        f = v.field(t, 4)
        instr = 0
        if f is not None:
            v.rng(f, 1)
            instr = v.b[f]
        f = v.field(t, 6)
        param = None
        if f is not None:
            p = v.follow(f)
            param = (p + 4, v.string(p))
        f = v.field(t, 8)
        sender = v.string(v.follow(f)) if f is not None else None
        f = v.field(t, 10)
        world = None
        if f is not None:
            p = v.follow(f)
            world = (p + 4, v.string(p))
        f = v.field(t, 12)
        repl = 0
        if f is not None:
            v.rng(f, 1)
            repl = v.b[f]
        n_rec, rec_dec = _tables(v, t, 14, False)
        n_ent, ent_dec = _tables(v, t, 16, True)
        f = v.field(t, 18)
        pos = None
        if f is not None:
            v.rng(f, 24)
            pos = struct.unpack_from("<3d", v.b, f)
        f = v.field(t, 20)
        if f is not None:
            p = v.follow(f)
            v.aligned(p, 4)
            v.vec(p, 1)
    except _Invalid:
        return {"status": INVALID_FLATBUFFER}
    if world is None or sender is None:
        return {"status": MISSING_FIELD}
    if rec_dec != OK:
        return {"status": rec_dec}
    if ent_dec != OK:
        return {"status": ent_dec}
    u = parse_uuid(sender)
    if u is None:
        return {"status": BAD_UUID}
    out.update(instruction=instr if instr <= 12 else 255, replication=repl if repl <= 2 else 0,
               sender_uuid=u, position=pos, world_off=world[0], world=world[1],
               parameter=None if param is None else param[1], n_records=n_rec, n_entities=n_ent)
    return out
