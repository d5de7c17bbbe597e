"""Seeded WorldQL Message frames for the wire-codec tests: valid frames over every field and
edge value the decoder reads, plus malformed ones (uuid forms, missing required fields, bad
UTF-8, missing NUL, truncations and random byte corruption)."""
from __future__ import annotations

import math
import random
import struct

from fbs_builder import message

UUIDS_OK = [
    "67e55044-10b1-426f-9247-bb680e5fe0c8",
    "67E55044-10B1-426F-9247-BB680E5FE0C8",
    "67e5504410b1426f9247bb680e5fe0c8",
    "urn:uuid:67e55044-10b1-426f-9247-bb680e5fe0c8",
    "00000000-0000-0000-0000-000000000000",
    "ffffffff-ffff-ffff-ffff-ffffffffffff",
]
UUIDS_BAD = [
    "", "67e55044", "67e55044-10b1-426f-9247-bb680e5fe0c", "67e55044-10b1-426f-9247-bb680e5fe0c8a",
    "{67e55044-10b1-426f-9247-bb680e5fe0c8}", "URN:UUID:67e55044-10b1-426f-9247-bb680e5fe0c8",
    "67e5504-410b1-426f-9247-bb680e5fe0c8", "67e55044-10b1-426f-9247bb680e5fe0c8-", "67e55044_10b1_426f_9247_bb680e5fe0c8",
    "g7e55044-10b1-426f-9247-bb680e5fe0c8", "67e5504410b1426f9247bb680e5fe0cg", "67e55044-10b1-426f-9247-bb680e5fe0-8",
    "-7e55044-10b1-426f-9247-bb680e5fe0c8", "67e55044-10b1-426f-9247-bb680e5fe0cé",
    "urn:uuid:67e5504410b1426f9247bb680e5fe0c8", "urn:uuid:67e55044-10b1-426f-9247-bb680e5fe0c8x",
]
WORLDS = ["world", "w00", "@global", "chat/server_1", "a b", "", "0bad", "été", "x" * 63, "x" * 70]
FLOATS = [0.0, -0.0, 1.5, -7.25, 16.0, -16.0, 1e308, -1e-308, 5e-324, math.inf, -math.inf, math.nan]


def _rand_uuid(r: random.Random) -> str:
    h = "%032x" % r.getrandbits(128)
    form = r.randrange(3)
    hy = f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"
    return hy if form == 0 else h if form == 1 else "urn:uuid:" + hy


def _record(r: random.Random, entity: bool, valid: bool) -> dict:
    d = dict(uuid=_rand_uuid(r), position=(r.uniform(-1e3, 1e3), 0.5, -2.0), world_name=r.choice(WORLDS[:2]),
             data=r.choice([None, "payload", ""]), flex=r.choice([None, b"\x01\x02\x03"]))
    if not entity and r.random() < 0.5:
        d["position"] = None  # optional for a Record
    if not valid:
        k = r.randrange(3)
        if k == 0:
            d["uuid"] = None
        elif k == 1:
            d["world_name"] = None
        else:
            d["uuid"] = r.choice(UUIDS_BAD)
        if entity and r.random() < 0.3:
            d["position"] = None
    return d


def valid_frame(r: random.Random, **over) -> bytes:
    f = dict(instruction=r.choice([None, 0, 4, 5, 6, 7, 7, 7, 12, 13, 200, 255]),
             parameter=r.choice([None, "p", "", "paramü"]),
             sender_uuid=r.choice(UUIDS_OK + [_rand_uuid(r)] * 4),
             world_name=r.choice(WORLDS), replication=r.choice([None, 0, 1, 2, 3, 255]),
             records=r.choice([None, [], [_record(r, False, True) for _ in range(r.randrange(1, 3))]]),
             entities=r.choice([None, [], [_record(r, True, True) for _ in range(r.randrange(1, 3))]]),
             position=r.choice([None, (r.uniform(-600, 600), r.uniform(-600, 600), r.uniform(-600, 600)),
                                tuple(r.choice(FLOATS) for _ in range(3))]),
             flex=r.choice([None, b"", b"\xff" * 5]))
    f.update(over)
    return message(**f)


def malformed_frame(r: random.Random) -> bytes:
    k = r.randrange(11)
    if k == 0:
        return valid_frame(r, sender_uuid=r.choice(UUIDS_BAD))
    if k == 1:
        return valid_frame(r, sender_uuid=None)
    if k == 2:
        return valid_frame(r, world_name=None)
    if k == 3:
        return valid_frame(r, world_name=b"bad\xff\xfeutf8")
    if k == 4:
        return valid_frame(r, records=[_record(r, False, False)])
    if k == 5:
        return valid_frame(r, entities=[_record(r, True, True), _record(r, True, False)])
    b = bytearray(valid_frame(r))
    if k == 6:  # truncation
        return bytes(b[:r.randrange(0, len(b))])
    if k == 7:  # strip the NUL after the last string (and its padding)
        return bytes(b.rstrip(b"\0"))
    if k == 8:  # root offset out of range / unaligned
        struct.pack_into("<I", b, 0, r.choice([len(b) + 4, 2, 0xFFFFFFFF]))
        return bytes(b)
    # k 9-10: random byte corruption
    for _ in range(r.randrange(1, 4)):
        i = r.randrange(len(b))
        b[i] = r.randrange(256)
    return bytes(b)


def cases(seed: int, n_valid: int, n_bad: int):
    r = random.Random(seed)
    frames = [valid_frame(r) for _ in range(n_valid)] + [malformed_frame(r) for _ in range(n_bad)]
    for u in UUIDS_OK + UUIDS_BAD:
        frames.append(message(instruction=7, sender_uuid=u, world_name="world", position=(1.0, 2.0, 3.0)))
    frames.append(b"")
    frames.append(b"\x04\0\0\0")
    return frames
