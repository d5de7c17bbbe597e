"""Minimal FlatBuffers writer for WorldQL Message frames (test helper).

Lays a frame out front to back — root uoffset, then each table preceded by its vtable, then the
table's children — which is a valid FlatBuffer (uoffsets point forward, soffsets back to the
vtable) though not byte-identical to the Rust builder's back-to-front layout. Field slots follow
worldql_server/src/flatbuffers/WorldQLFB_generated.rs: Message :939-947, Record/Entity :485-489 /
:704-708; Vec3d = three little-endian f64 (:254-257).
"""
from __future__ import annotations

import struct
from typing import Optional, Sequence

MESSAGE_SLOTS = ["instruction", "parameter", "sender_uuid", "world_name", "replication", "records",
                 "entities", "position", "flex"]
RECORD_SLOTS = ["uuid", "position", "world_name", "data", "flex"]
KINDS = {"instruction": "u8", "replication": "u8", "position": "vec3", "flex": "bytes",
         "records": "tables", "entities": "tables"}  # everything else: string


class _W:
    def __init__(self):
        self.b = bytearray()

    def pad(self, a):
        while len(self.b) % a:
            self.b.append(0)

    def table(self, slots, fields: dict):
        """Append vtable + table for `fields` (slot name -> value); children after it."""
        present = [s for s in slots if fields.get(s) is not None]
        # inline layout: [soffset][uoffset slots][vec3 (8-aligned)][u8 scalars]
        layout, off = {}, 4
        for s in present:
            if KINDS.get(s, "str") in ("str", "bytes", "tables"):
                layout[s] = off
                off += 4
        if "position" in present:
            off = (off + 7) // 8 * 8
            layout["position"] = off
            off += 24
        for s in present:
            if KINDS.get(s) == "u8":
                layout[s] = off
                off += 1
        tbl_len = off
        vt_len = 4 + 2 * len(slots)
        self.pad(2)
        vt_pos = len(self.b)
        self.b += struct.pack("<HH", vt_len, tbl_len)
        for s in slots:
            self.b += struct.pack("<H", layout.get(s, 0))
        # the table: 8-aligned start so the Vec3d inside it is naturally aligned
        while (len(self.b) % 8) != 0:
            self.b.append(0)
        t_pos = len(self.b)
        self.b += b"\0" * tbl_len
        struct.pack_into("<i", self.b, t_pos, t_pos - vt_pos)
        for s in present:
            k, v = KINDS.get(s, "str"), fields[s]
            if k == "u8":
                self.b[t_pos + layout[s]] = v & 0xFF
            elif k == "vec3":
                struct.pack_into("<3d", self.b, t_pos + layout[s], *v)
        for s in present:  # children, in slot order
            k, v = KINDS.get(s, "str"), fields[s]
            slot = t_pos + layout[s]
            if k == "str":
                self._string(slot, v.encode("utf-8") if isinstance(v, str) else bytes(v))
            elif k == "bytes":
                self._string(slot, bytes(v), nul=False)
            elif k == "tables":
                self.pad(4)
                vpos = len(self.b)
                struct.pack_into("<I", self.b, slot, vpos - slot)
                self.b += struct.pack("<I", len(v)) + b"\0" * (4 * len(v))
                for i, rec in enumerate(v):
                    tp = self.table(RECORD_SLOTS, rec)
                    eslot = vpos + 4 + 4 * i
                    struct.pack_into("<I", self.b, eslot, tp - eslot)
        return t_pos

    def _string(self, slot, raw: bytes, nul=True):
        self.pad(4)
        p = len(self.b)
        struct.pack_into("<I", self.b, slot, p - slot)
        self.b += struct.pack("<I", len(raw)) + raw + (b"\0" if nul else b"")


def message(instruction: Optional[int] = None, parameter=None, sender_uuid=None, world_name=None,
            replication: Optional[int] = None, records: Optional[Sequence[dict]] = None,
            entities: Optional[Sequence[dict]] = None, position=None, flex=None) -> bytes:
    """One Message frame; a field left None is absent from the frame."""
    fields = dict(instruction=instruction, parameter=parameter, sender_uuid=sender_uuid,
                  world_name=world_name, replication=replication, records=records, entities=entities,
                  position=position, flex=flex)
    w = _W()
    w.b += b"\0\0\0\0"  # root uoffset
    t = w.table(MESSAGE_SLOTS, fields)
    struct.pack_into("<I", w.b, 0, t)
    w.pad(4)
    return bytes(w.b)
