"""Host wire codec: the C++ batch decoder / sanitizer of libwq_router.so
against the Python restatement oracle/fbs_oracle.py, the committed golden frames, the frames'
own field values, and the reference's sanitize_world_name unit-test vectors. CPU only."""
import json
import math
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

from fbs_builder import message  # noqa: E402
from fbs_cases import UUIDS_BAD, UUIDS_OK, cases, valid_frame  # noqa: E402
from oracle import fbs_oracle  # noqa: E402

codec = pytest.importorskip("worldql_server_amd.codec")
GOLDEN = os.path.join(HERE, "golden", "fbs_frames.npz")


def _same_pos(a, b):
    return all((math.isnan(x) and math.isnan(y)) or (struct.pack("<d", x) == struct.pack("<d", y))
               for x, y in zip(a, b))


def _check_against_oracle(frames, recs):
    for i, (f, r) in enumerate(zip(frames, recs)):
        d = fbs_oracle.decode(f)
        assert r["status"] == d["status"], (i, f, d)
        if d["status"] != 0:
            continue
        assert r["instruction"] == d["instruction"]
        assert r["replication"] == d["replication"]
        assert bytes(r["sender_uuid"]) == d["sender_uuid"]
        assert bool(r["has_position"]) == (d["position"] is not None)
        if d["position"] is not None:
            assert _same_pos(r["position"], d["position"])
        w0, wl = int(r["world_off"]), int(r["world_len"])
        assert w0 == d["world_off"] and f[w0:w0 + wl] == d["world"]
        assert bool(r["has_parameter"]) == (d["parameter"] is not None)
        assert r["n_records"] == d["n_records"] and r["n_entities"] == d["n_entities"]


def test_golden_frames_oracle_and_codec():
    g = np.load(GOLDEN)
    data, offsets = g["data"], g["offsets"]
    frames = [bytes(data[offsets[i]:offsets[i + 1]]) for i in range(len(offsets) - 1)]
    # the restatement still reproduces its committed outputs
    for i, f in enumerate(frames):
        assert fbs_oracle.decode(f)["status"] == g["status"][i]
    recs = codec.decode_packed(data, offsets)
    for k in ("status", "instruction", "replication", "has_position", "world_off", "world_len",
              "n_records", "n_entities"):
        np.testing.assert_array_equal(recs[k].astype(np.uint32), g[k], err_msg=k)
    np.testing.assert_array_equal(recs["sender_uuid"], g["sender_uuid"])
    keep = ~np.isnan(g["position"])
    np.testing.assert_array_equal(recs["position"].view(np.uint64)[keep], g["position"].view(np.uint64)[keep])
    assert (g["status"] == 0).sum() > 100 and len(set(g["status"].tolist())) == 4


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_frames_match_oracle(seed):
    frames = cases(seed, 400, 600)
    _check_against_oracle(frames, codec.decode_batch(frames))


def test_valid_frames_carry_their_fields():
    r = random.Random(7)
    for _ in range(300):
        sender = str(uuid.UUID(int=r.getrandbits(128)))
        pos = (r.uniform(-1e4, 1e4), -0.0, r.choice([math.inf, 5e-324, 3.0]))
        instr, repl = r.choice([4, 5, 7, 6, 30]), r.choice([0, 1, 2, 9])
        world = r.choice(["world", "w42", "chat/server_1", "ünïcode"])
        f = valid_frame(r, instruction=instr, sender_uuid=sender, position=pos, replication=repl, world_name=world)
        rec = codec.decode_batch([f])[0]
        assert rec["status"] == codec.DEC_OK
        assert rec["instruction"] == (instr if instr <= 12 else 255)
        assert rec["replication"] == (repl if repl <= 2 else 0)
        assert bytes(rec["sender_uuid"]) == uuid.UUID(sender).bytes
        assert _same_pos(rec["position"], pos)
        w0, wl = int(rec["world_off"]), int(rec["world_len"])
        assert f[w0:w0 + wl].decode("utf-8") == world


def test_uuid_forms():
    for u in UUIDS_OK:
        rec = codec.decode_batch([message(instruction=7, sender_uuid=u, world_name="world")])[0]
        assert rec["status"] == codec.DEC_OK, u
        assert bytes(rec["sender_uuid"]) == uuid.UUID(u.replace("urn:uuid:", "")).bytes
    for u in UUIDS_BAD:
        rec = codec.decode_batch([message(instruction=7, sender_uuid=u, world_name="world")])[0]
        assert rec["status"] == codec.DEC_BAD_UUID, u


def test_missing_fields_and_defaults():
    u = UUIDS_OK[0]
    recs = codec.decode_batch([
        message(sender_uuid=u, world_name="w"),               # defaults: Heartbeat, ExceptSelf
        message(instruction=7, world_name="w"),               # no sender
        message(instruction=7, sender_uuid=u),                # no world
        message(instruction=7, sender_uuid=u, world_name="w", entities=[dict(uuid=u, world_name="w")]),
        message(instruction=7, sender_uuid=u, world_name="w", records=[dict(uuid=u, world_name="w")]),
    ])
    assert recs["status"].tolist() == [0, 2, 2, 2, 0]
    assert recs[0]["instruction"] == 0 and recs[0]["replication"] == 0 and recs[0]["has_position"] == 0
    assert recs[4]["n_records"] == 1


def test_corrupt_and_empty_frames_never_crash():
    r = random.Random(11)
    frames = [b"", b"\0", b"\xff" * 3, b"\x04\0\0\0\x00\x00"]
    base = valid_frame(r)
    for n in range(len(base)):
        frames.append(base[:n])  # every strict truncation
    recs = codec.decode_batch(frames)
    assert (recs["status"] == codec.DEC_INVALID_FLATBUFFER).all()
    _check_against_oracle(frames, recs)


def test_threaded_decode_matches_single_thread():
    frames = cases(5, 5000, 5000)
    a = codec.decode_batch(frames, n_threads=1)
    b = codec.decode_batch(frames, n_threads=8)
    assert a.tobytes() == b.tobytes()


def test_decode_messages_events():
    from worldql_server_amd.processing import LOCAL_MESSAGE
    u = UUIDS_OK[0]
    frames = [message(instruction=7, sender_uuid=u, world_name="world", position=(1.0, 2.0, 3.0), replication=1),
              message(instruction=7, sender_uuid="nope", world_name="world"),
              message(instruction=4, sender_uuid=u, world_name="chat/server_1")]
    ev = codec.decode_messages(frames)
    assert ev[1] is None
    assert ev[0].instruction == LOCAL_MESSAGE and ev[0].world_name == "world" and ev[0].replication == 1
    assert ev[0].sender_uuid == uuid.UUID(u) and (ev[0].position.x, ev[0].position.y, ev[0].position.z) == (1, 2, 3)
    assert ev[2].instruction == "AreaSubscribe" and ev[2].position is None


def test_sanitize_reference_vectors():
    kats = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))
    for raw, want in kats["sanitize_ok"]:
        assert codec.sanitize_world_name(raw) == want
    for raw, kind in kats["sanitize_err"]:
        with pytest.raises(codec.SanitizeCError) as e:
            codec.sanitize_world_name(raw)
        assert e.value.kind == kind, raw


def test_sanitize_matches_python_restatement():
    from worldql_server_amd.world_names import SanitizeError, sanitize_world_name
    r = random.Random(3)
    alphabet = "abcXYZ09_ /\\:@-é€\u0000"
    for _ in range(3000):
        s = "".join(r.choice(alphabet) for _ in range(r.randrange(0, 30)))
        try:
            want = sanitize_world_name(s)
        except SanitizeError as e:
            with pytest.raises(codec.SanitizeCError) as got:
                codec.sanitize_world_name(s)
            assert got.value.kind == e.kind, s
            continue
        assert codec.sanitize_world_name(s) == want
