"""Generates tests/golden/fbs_frames.npz: WorldQL Message frames (tests/fbs_cases.py, seed 0xF4)
and what Message::deserialize returns for each, by the Python restatement oracle/fbs_oracle.py.
Run from the repo root: python tests/golden/make_fbs_golden.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from fbs_cases import cases  # noqa: E402
from oracle import fbs_oracle  # noqa: E402


def expected(frames):
    n = len(frames)
    e = {k: np.zeros(n, np.uint32) for k in ("status", "instruction", "replication", "has_position",
                                              "world_off", "world_len", "n_records", "n_entities")}
    e["position"] = np.zeros((n, 3), np.float64)
    e["sender_uuid"] = np.zeros((n, 16), np.uint8)
    for i, f in enumerate(frames):
        d = fbs_oracle.decode(f)
        e["status"][i] = d["status"]
        if d["status"] != fbs_oracle.OK:
            continue
        e["instruction"][i] = d["instruction"]
        e["replication"][i] = d["replication"]
        e["has_position"][i] = d["position"] is not None
        if d["position"] is not None:
            e["position"][i] = d["position"]
        e["sender_uuid"][i] = np.frombuffer(d["sender_uuid"], np.uint8)
        e["world_off"][i] = d["world_off"]
        e["world_len"][i] = len(d["world"])
        e["n_records"][i] = d["n_records"]
        e["n_entities"][i] = d["n_entities"]
    return e


def main():
    frames = cases(0xF4, 300, 300)
    offsets = np.zeros(len(frames) + 1, np.uint64)
    offsets[1:] = np.cumsum([len(f) for f in frames])
    data = np.frombuffer(b"".join(frames), np.uint8)
    e = expected(frames)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fbs_frames.npz")
    np.savez_compressed(out, data=data, offsets=offsets, **e)
    print(out, len(frames), "frames,", int((e["status"] == 0).sum()), "decode OK")


if __name__ == "__main__":
    main()
