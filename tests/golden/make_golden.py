"""Generates the golden fixtures under tests/golden/.

1. reference_kats.json — the reference's own unit-test vectors, transcribed as data:
   cube_area.rs:102-142 (coord_clamp_10 / coord_clamp_8), cube_area.rs:156-175 (from_vector3),
   round.rs:28-76 (round_positive / round_negative), area_map.rs:154-254 (area_subscriptions /
   world_subscriptions as op sequences with expected membership), world_names.rs:127-171
   (sanitize). These pin the restatements (the Rust reference cannot be built: SURVEY.md §8(c)).
2. quantize_edges.json — Appendix A.3 edge floats (NaN, +-inf, +-0, denormals, 2^63 ...) at the
   sizes {1,3,8,10,16,17,100,65535}, expected values from the numpy restatement, which must
   first reproduce every KAT of (1) and agree with the C restatement.
3. quantize_random.npz — random f64 bit patterns (all exponent ranges) plus uniform coordinates
   per size, same provenance as (2).
4. routing_cases.npz — small routing scenarios (worlds, replication modes, churn sequences,
   raw off-grid keys, sender not subscribed, remove_peer) with the C restatement's output.

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as orc  # noqa: E402
from worldql_server_amd import abi  # noqa: E402
from worldql_server_amd.synth import SplitMix64  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SIZES = [1, 3, 8, 10, 16, 17, 100, 65535]

# --- (1) reference KATs, transcribed -------------------------------------------------------
COORD_CLAMP = [  # cube_area.rs:102-121 (size 10), :123-142 (size 8)
    [0.0, 10, 10], [0.1, 10, 10], [5.0, 10, 10], [9.99999, 10, 10], [10.0, 10, 10], [10.1, 10, 20],
    [-0.1, 10, -10], [-5.0, 10, -10], [-9.99999, 10, -10], [-10.0, 10, -10], [-10.1, 10, -20],
    [-20.0, 10, -20],
    [0.0, 8, 8], [0.1, 8, 8], [5.0, 8, 8], [9.99999, 8, 16], [10.0, 8, 16], [10.1, 8, 16],
    [-0.1, 8, -8], [-5.0, 8, -8], [-9.99999, 8, -16], [-10.0, 8, -16], [-10.1, 8, -16],
    [-20.0, 8, -24],
]
FROM_VECTOR3 = [  # cube_area.rs:156-175, size 10
    [[0.0, 0.0, 0.0], 10, [10, 10, 10]],
    [[0.1, 0.3, 2.5], 10, [10, 10, 10]],
    [[3.0, 4.0, 5.0], 10, [10, 10, 10]],
    [[9.1, 9.9, 9.9], 10, [10, 10, 10]],
    [[18.0, 12.5, 16.7], 10, [20, 20, 20]],
    [[-3.0, -8.0, -1.3], 10, [-10, -10, -10]],
    [[-6.0, -0.3, -9.9], 10, [-10, -10, -10]],
    [[-12.0, -19.9, -13.5], 10, [-20, -20, -20]],
    [[25.0, -13.2, 0.0], 10, [30, -20, 10]],
    [[25.0, -13.2, -0.1], 10, [30, -20, -10]],
]
ROUND_BY_MULTIPLE = [  # round.rs:28-54 (round_positive), :56-76 (round_negative)
    [0.0, 10.0, 10.0], [-0.0, 10.0, 10.0], [0.1, 10.0, 10.0], [1.0, 10.0, 10.0], [5.0, 10.0, 10.0],
    [9.0, 10.0, 10.0], [9.0, 10.0, 10.0], [9.9999, 10.0, 10.0], [10.0, 10.0, 10.0],
    [10.0001, 10.0, 20.0], [15.0, 10.0, 20.0], [20.0, 10.0, 20.0],
    [0.0, 8.0, 8.0], [-0.0, 8.0, 8.0], [2.0, 8.0, 8.0], [5.0, 8.0, 8.0], [7.0, 8.0, 8.0],
    [8.0, 8.0, 8.0], [9.0, 8.0, 16.0], [15.0, 8.0, 16.0], [16.0, 8.0, 16.0],
    [-1.0, 10.0, 0.0], [-5.0, 10.0, 0.0], [-9.0, 10.0, 0.0], [-9.0, 10.0, 0.0], [-9.9999, 10.0, 0.0],
    [-10.0, 10.0, -10.0], [-10.0001, 10.0, -10.0], [-15.0, 10.0, -10.0], [-20.0, 10.0, -20.0],
    [-2.0, 8.0, 0.0], [-5.0, 8.0, 0.0], [-7.0, 8.0, 0.0], [-8.0, 8.0, -8.0], [-15.0, 8.0, -8.0],
    [-16.0, 8.0, -16.0],
]
C1 = {"raw": [0, 0, 0]}
C2 = {"raw": [16, 16, 16]}
V1 = {"pos": [6.3, 1.0, 10.5]}  # "Equivalent to cube_2" (area_map.rs:162-163)
AREA_SUBSCRIPTIONS = {  # area_map.rs:154-205, one peer "u", AreaMap::new(16, "world")
    "cube_size": 16,
    "steps": [
        {"op": None, "expect": [["u", C1, False], ["u", C2, False], ["u", V1, False]]},
        {"op": ["add", "u", C1], "expect": [["u", C1, True], ["u", C2, False], ["u", V1, False]]},
        {"op": ["add", "u", C2], "expect": [["u", C1, True], ["u", C2, True], ["u", V1, True]]},
        {"op": ["remove", "u", C1], "expect": [["u", C1, False], ["u", C2, True], ["u", V1, True]]},
        {"op": ["remove", "u", C2], "expect": [["u", C1, False], ["u", C2, False], ["u", V1, False]]},
        {"op": ["add", "u", V1], "expect": [["u", C1, False], ["u", C2, True], ["u", V1, True]]},
        {"op": ["remove", "u", V1], "expect": [["u", C1, False], ["u", C2, False], ["u", V1, False]]},
    ],
}
WORLD_SUBSCRIPTIONS = {  # area_map.rs:207-254, is_peer_subscribed_any after each step
    "cube_size": 16,
    "steps": [
        {"op": None, "expect_any": [["u1", False], ["u2", False]]},
        {"op": ["add", "u1", C1], "expect_any": [["u1", True], ["u2", False]]},
        {"op": ["add", "u1", C2], "expect_any": [["u1", True], ["u2", False]]},
        {"op": ["add", "u2", C2], "expect_any": [["u1", True], ["u2", True]]},
        {"op": ["remove", "u1", C1], "expect_any": [["u1", True], ["u2", True]]},
        {"op": ["remove", "u1", C2], "expect_any": [["u1", False], ["u2", True]]},
        {"op": ["add", "u2", C1], "expect_any": [["u1", False], ["u2", True]]},
        {"op": ["remove_peer", "u2", None], "expect_any": [["u1", False], ["u2", False]]},
    ],
}
SANITIZE_OK = [  # world_names.rs:127-141
    ["world", "world"], ["WORLD", "WORLD"], ["world_1_2_3", "world_1_2_3"], ["world one", "world_one"],
    ["chat/server_1", "chat_fs_server_1"], ["chat\\server_2", "chat_bs_server_2"],
    ["chat:server_3", "chat_cl_server_3"], ["chat@server_4", "chat_at_server_4"],
    ["a" * 63, "a" * 63],
]
SANITIZE_ERR = [  # world_names.rs:143-170
    ["@global", "IsGlobalWorld"], ["", "ZeroLength"],
    ["0world", "InvalidStart"], ["_world", "InvalidStart"], ["/world", "InvalidStart"],
    ["\\world", "InvalidStart"], [":world", "InvalidStart"], ["@world", "InvalidStart"],
    [" world", "InvalidStart"], ["[world", "InvalidStart"], ["]world", "InvalidStart"],
    ["world (two)", "InvalidChars"], ["world&three", "InvalidChars"], ["world*four", "InvalidChars"],
    ["world-four", "InvalidChars"],
    ["a" * 64, "TooLong"],
]

# Appendix A.3 edge inputs (values are computed, not transcribed)
EDGE_INPUTS = [
    0.0, -0.0, 16.0, -16.0, 10.0, -10.0, 15.999999999999998, -15.999999999999998,
    16.000000000000004, -16.000000000000004, 5e-324, -5e-324, 2.2250738585072014e-308,
    -2.2250738585072014e-308, 1e-310, -1e-310, float("nan"), float("inf"), float("-inf"),
    1e300, -1e300, 2.0 ** 63, -(2.0 ** 63), 2.0 ** 63 - 1024.0, -(2.0 ** 63) + 1024.0,
    2.0 ** 52, 2.0 ** 52 + 1.0, 2.0 ** 53 + 2.0, -(2.0 ** 53) - 2.0, 1.7976931348623157e308,
    -1.7976931348623157e308, 0.5, -0.5, 1.0, -1.0, 65535.0, -65535.0, 65536.0, 131070.0,
    -131070.0, 1e-5, -1e-5, 123456.789, -123456.789, 9.99999, -9.99999,
]


def check_restatements() -> None:
    """Both restatements must reproduce every reference KAT before anything is emitted."""
    for c, s, e in COORD_CLAMP:
        assert int(orc.coord_clamp_np(c, s)) == e, (c, s, e)
        assert int(orc.c_coord_clamp(np.array([c]), s)[0]) == e, (c, s, e)
    for p, s, e in FROM_VECTOR3:
        assert orc.quantize_np(p, s).tolist() == e, (p, e)
        assert orc.c_coord_clamp(np.array(p), s).tolist() == e, (p, e)
    lib = orc.load_c_oracle()
    for n, m, e in ROUND_BY_MULTIPLE:
        assert float(orc.round_by_multiple_np(n, m)) == e, (n, m, e)
        assert lib.wqo_round_by_multiple(n, m) == e, (n, m, e)


def random_bit_patterns(rng: SplitMix64, n: int) -> np.ndarray:
    bits = rng.next_u64(n)
    x = bits.view(np.float64).copy()
    # add scaled "ordinary" coordinates so the common regime is well covered
    u = rng.uniform(-5000.0, 5000.0, n)
    x[: n // 2] = u[: n // 2]
    return x


def routing_cases() -> dict:
    """Small routing scenarios; expected output from the C restatement."""
    out = {}
    rng = SplitMix64(0x5EED00FF)
    case_id = 0
    for cube_size in (16, 10, 7):
        for n_worlds in (1, 3):
            ops = []
            n_peers = 40
            # subscriptions: each peer subscribes a few cubes around a random point, some by raw key
            for p in range(n_peers):
                w = int(rng.next_u64(1)[0] % n_worlds)
                c = rng.uniform(-40.0, 40.0, 3)
                for d in range(int(rng.next_u64(1)[0] % 4) + 1):
                    jitter = rng.uniform(-cube_size, cube_size, 3)
                    if rng.next_u64(1)[0] % 5 == 0:
                        key = orc.quantize_np(c + jitter, cube_size)
                        if rng.next_u64(1)[0] % 3 == 0:
                            key = key + 1  # off-grid raw key, unreachable from any Vector3
                        ops.append(abi.make_op(w, p, abi.OP_SUBSCRIBE, key=key))
                    else:
                        ops.append(abi.make_op(w, p, abi.OP_SUBSCRIBE, pos=c + jitter))
            # churn: unsubscribes (some of absent subscriptions), re-subscribes, disconnects
            for i in range(60):
                p = int(rng.next_u64(1)[0] % n_peers)
                w = int(rng.next_u64(1)[0] % n_worlds)
                k = int(rng.next_u64(1)[0] % 10)
                pos = rng.uniform(-40.0, 40.0, 3)
                if k < 5:
                    ops.append(abi.make_op(w, p, abi.OP_UNSUBSCRIBE, pos=pos))
                elif k < 9:
                    ops.append(abi.make_op(w, p, abi.OP_SUBSCRIBE, pos=pos))
                elif i % 2:
                    ops.append(abi.make_op(abi.WORLD_INVALID, p, abi.OP_REMOVE_PEER, pos=pos))  # WorldMap
                else:
                    ops.append(abi.make_op(w, p, abi.OP_REMOVE_PEER, pos=pos))  # AreaMap, one world
            # unsubscribe exactly what an earlier op subscribed (exercise real removals)
            for o in list(ops[:30]):
                if o["kind"] == abi.OP_SUBSCRIBE and rng.next_u64(1)[0] % 2 == 0:
                    o2 = o.copy()
                    o2["kind"] = abi.OP_UNSUBSCRIBE
                    ops.append(o2)
            ops = np.array(ops, dtype=abi.OP_DTYPE)
            M = 400
            pos = rng.uniform(-48.0, 48.0, 3 * M).reshape(M, 3)
            pos[::7] = orc.quantize_np(pos[::7], cube_size).astype(np.float64)  # exact multiples
            pos[3::11] = 0.0
            world = (rng.next_u64(M) % np.uint64(n_worlds + 1)).astype(np.uint32)  # one unknown world
            sender = (rng.next_u64(M) % np.uint64(n_peers + 2)).astype(np.uint32)
            repl = (rng.next_u64(M) % np.uint64(4)).astype(np.uint8)  # 3 = unknown -> ExceptSelf
            o = orc.COracle(cube_size)
            o.apply_ops(ops)
            offs, peers, F = o.route(pos, world, sender, repl)
            pre = f"c{case_id}_"
            out.update({pre + "cube_size": np.array([cube_size]), pre + "ops": ops.view(np.uint8),
                        pre + "pos": pos, pre + "world": world, pre + "sender": sender, pre + "repl": repl,
                        pre + "offsets": offs, pre + "peers": peers, pre + "F": np.array([F], dtype=np.uint64)})
            case_id += 1
    out["n_cases"] = np.array([case_id])
    return out


def main() -> None:
    check_restatements()
    kats = {
        "source": "Transcribed from the reference's #[test] functions (paths relative to "
                  "worldql_server/src/): subscriptions/cube_area.rs:102-175, utils/round.rs:28-76, "
                  "subscriptions/area_map.rs:154-254, utils/world_names.rs:127-171.",
        "coord_clamp": COORD_CLAMP,
        "from_vector3": FROM_VECTOR3,
        "round_by_multiple": ROUND_BY_MULTIPLE,
        "area_subscriptions": AREA_SUBSCRIPTIONS,
        "world_subscriptions": WORLD_SUBSCRIPTIONS,
        "sanitize_ok": SANITIZE_OK,
        "sanitize_err": SANITIZE_ERR,
    }
    with open(os.path.join(OUT, "reference_kats.json"), "w") as f:
        json.dump(kats, f, indent=1)

    edges = []
    x = np.array(EDGE_INPUTS, dtype=np.float64)
    for s in SIZES:
        py = orc.coord_clamp_np(x, s)
        c = orc.c_coord_clamp(x, s)
        assert (py == c).all(), s
        for xi, e in zip(x.tolist(), py.tolist()):
            edges.append([repr(xi), s, int(e)])
    with open(os.path.join(OUT, "quantize_edges.json"), "w") as f:
        json.dump({"note": "coord floats as Python repr strings (nan/inf safe); expected from "
                           "oracle/oracle.py coord_clamp_np == oracle/wq_oracle.c", "vectors": edges}, f)

    rng = SplitMix64(0x5EED0A11)
    arrs = {}
    for s in SIZES:
        xs = random_bit_patterns(rng, 4096)
        py = orc.coord_clamp_np(xs, s)
        c = orc.c_coord_clamp(xs, s)
        assert (py == c).all(), s
        arrs[f"x_{s}"] = xs
        arrs[f"k_{s}"] = py
    np.savez_compressed(os.path.join(OUT, "quantize_random.npz"), **arrs)

    np.savez_compressed(os.path.join(OUT, "routing_cases.npz"), **routing_cases())
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
