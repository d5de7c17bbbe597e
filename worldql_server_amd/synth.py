"""Deterministic synthetic workloads, reproducible in C++ and Python.

RNG: splitmix64; f64 uniform draw = lo + (hi - lo) * ((u >> 11) * 2^-53); Gaussian = Box–Muller
from two such draws. Seeds are 0x5EED0000 + config number. Each logical stream (peer positions,
message positions, senders, ...) has its own generator seeded from (config seed, stream id), so a
stream does not depend on how many draws other streams made.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import abi

GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


class SplitMix64:
    def __init__(self, seed: int):
        self.state = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)

    def next_u64(self, n: int) -> np.ndarray:
        with np.errstate(over="ignore"):
            z = self.state + GAMMA * np.arange(1, n + 1, dtype=np.uint64)
            self.state = self.state + GAMMA * np.uint64(n)
        return _mix(z)

    def uniform(self, lo: float, hi: float, n: int) -> np.ndarray:
        u = (self.next_u64(n) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
        return lo + (hi - lo) * u

    def below(self, bound: int, n: int) -> np.ndarray:
        return (self.next_u64(n) % np.uint64(bound)).astype(np.uint32)

    def normal(self, n: int) -> np.ndarray:
        u1 = self.uniform(0.0, 1.0, n)
        u2 = self.uniform(0.0, 1.0, n)
        u1 = np.where(u1 <= 0.0, 2.0 ** -53, u1)
        return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def stream(config: int, stream_id: int) -> SplitMix64:
    seed = int(_mix(np.array([np.uint64(0x5EED0000 + config) ^ np.uint64(stream_id * 0x1000193)]))[0])
    return SplitMix64(seed)


NEIGHBOURHOOD = np.array([(dx, dy, dz) for dx in (-1, 0, 1) for dy in (-1, 0, 1) for dz in (-1, 0, 1)],
                         dtype=np.float64)


@dataclass
class Workload:
    name: str
    cube_size: int
    ops: np.ndarray          # wq_op records (subscriptions), applied once before routing
    pos: np.ndarray          # (M, 3) f64 message positions
    world: np.ndarray        # (M,) u32
    sender: np.ndarray       # (M,) u32
    repl: np.ndarray         # (M,) u8
    n_peers: int


def uniform_box(config: int, n_peers: int, n_msgs: int, half: float, neighbourhood: bool,
                cube_size: int = 16, repl_mode: str = "except", n_worlds: int = 1,
                world_offset: int = 0) -> Workload:
    """C1 / C2 shaped workload: uniform peers and messages in [-half, half)^3."""
    peer_pos = stream(config, 1).uniform(-half, half, 3 * n_peers).reshape(n_peers, 3)
    peer_world = (stream(config, 6).below(n_worlds, n_peers) if n_worlds > 1
                  else np.zeros(n_peers, dtype=np.uint32)) + np.uint32(world_offset)
    if neighbourhood:
        sub_pos = (peer_pos[:, None, :] + cube_size * NEIGHBOURHOOD[None, :, :]).reshape(-1, 3)
        sub_peer = np.repeat(np.arange(n_peers, dtype=np.uint32), 27)
        sub_world = np.repeat(peer_world, 27)
    else:
        sub_pos, sub_peer, sub_world = peer_pos, np.arange(n_peers, dtype=np.uint32), peer_world
    ops = abi.ops_array(sub_world, sub_peer, np.zeros(len(sub_peer), np.uint8), pos=sub_pos)
    pos = stream(config, 2).uniform(-half, half, 3 * n_msgs).reshape(n_msgs, 3)
    sender = stream(config, 3).below(n_peers, n_msgs)
    world = peer_world[sender] if n_worlds > 1 else np.full(n_msgs, world_offset, dtype=np.uint32)
    if repl_mode == "except":
        repl = np.zeros(n_msgs, dtype=np.uint8)
    else:
        repl = stream(config, 4).below(3, n_msgs).astype(np.uint8)
    return Workload(f"C{config}", cube_size, ops, pos, world.astype(np.uint32), sender, repl, n_peers)


def config_c1(repl_mode: str = "except") -> Workload:
    """C1: 1 world, 1k peers x 1 cube, 10k messages, U[-64,64)^3, cube_size 16."""
    return uniform_box(1, 1_000, 10_000, 64.0, neighbourhood=False, repl_mode=repl_mode)


def config_c2(repl_mode: str = "except", scale: float = 1.0, world_offset: int = 0) -> Workload:
    """C2: 1 world, 100k peers x 3x3x3 cubes, 1M messages, U[-512,512)^3, cube_size 16.

    `scale` shrinks peers, messages and the box volume together (fan-out preserved) for tests."""
    n_peers = max(1, int(round(100_000 * scale)))
    n_msgs = max(1, int(round(1_000_000 * scale)))
    half = 512.0 * (scale ** (1.0 / 3.0))
    return uniform_box(2, n_peers, n_msgs, half, neighbourhood=True, repl_mode=repl_mode,
                       world_offset=world_offset)
