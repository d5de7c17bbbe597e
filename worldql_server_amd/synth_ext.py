"""Synthetic workloads for SURVEY.md §8(d) C3 / C4 / C5 (same RNG conventions as synth.py).

C3  1M peers / 10M messages, 90% from 256 Gaussian hotspots (sigma 128, centres U[-4096,4096)^3,
    Zipf(1.0) weights), 10% uniform U[-4096,4096)^3; 3x3x3 subscriptions; cube-hash sharded.
C4  64 worlds x 50k peers, 3x3x3 each, box U[-256,256)^3 per world; per tick 5% of the peers move
    by N(0,16)^3 and emit AreaUnsubscribe for the cells they left and AreaSubscribe for the cells
    they entered; one message per peer at its own position (the sender is subscribed to its own
    cube, so ExceptSelf matters).
C5  N = M = 1M entities in U[-1024,1024)^3 with velocity U[-4,4)^3 per tick; each subscribes its
    3x3x3 and sends one message; exact radius filter r = 16 after the cube broadphase.

`scale` shrinks peer and message counts and the box volume together (occupancy and fan-out are
preserved) for tests; 1.0 is the configuration BASELINE.json names.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import abi
from .synth import NEIGHBOURHOOD, Workload, stream


def cell_keys(pos: np.ndarray, s: int) -> np.ndarray:
    """CubeArea of finite positions (cube_area.rs:23-44 for finite values: away from zero to a
    multiple of s, exact multiples kept, 0 -> s). Generator-side only: used to decide which cells a
    moving peer left / entered; the table itself always quantises on the GPU."""
    a = np.abs(pos)
    k = np.ceil(a / s) * s
    k = np.where(a == 0.0, float(s), k)
    return (np.where(pos < 0.0, -k, k)).astype(np.int64)


def _neighbourhood_ops(world: np.ndarray, peer_pos: np.ndarray, cube_size: int, peers=None,
                       kind: int = abi.OP_SUBSCRIBE) -> np.ndarray:
    n = len(peer_pos)
    peers = np.arange(n, dtype=np.uint32) if peers is None else np.asarray(peers, dtype=np.uint32)
    sub_pos = (peer_pos[:, None, :] + cube_size * NEIGHBOURHOOD[None, :, :]).reshape(-1, 3)
    return abi.ops_array(np.repeat(np.asarray(world, np.uint32), 27), np.repeat(peers, 27),
                         np.full(27 * n, kind, np.uint8), pos=sub_pos)


def hotspot_positions(config: int, stream_id: int, n: int, half: float, n_hot: int, sigma: float,
                      frac_hot: float = 0.9) -> np.ndarray:
    """n positions: frac_hot of them Gaussian around n_hot Zipf(1.0)-weighted centres, the rest
    uniform in [-half, half)^3. The centres have their own stream (shared by peers and messages)."""
    centres = stream(config, 100).uniform(-half, half, 3 * n_hot).reshape(n_hot, 3)
    w = 1.0 / np.arange(1, n_hot + 1, dtype=np.float64)
    cdf = np.cumsum(w / w.sum())
    g = stream(config, stream_id)
    hot = g.uniform(0.0, 1.0, n) < frac_hot
    pick = np.minimum(np.searchsorted(cdf, g.uniform(0.0, 1.0, n), side="right"), n_hot - 1)
    gauss = np.stack([g.normal(n), g.normal(n), g.normal(n)], 1) * sigma + centres[pick]
    unif = g.uniform(-half, half, 3 * n).reshape(n, 3)
    return np.where(hot[:, None], gauss, unif)


def config_c3(scale: float = 1.0, sigma: float = 128.0) -> Workload:
    """C3: 1M peers x 3x3x3, 10M messages, 256 Zipf-weighted Gaussian hotspots (90%) + uniform (10%)."""
    n_peers = max(1, int(round(1_000_000 * scale)))
    n_msgs = max(1, int(round(10_000_000 * scale)))
    half = 4096.0 * (scale ** (1.0 / 3.0))
    s = sigma * (scale ** (1.0 / 3.0))
    peer_pos = hotspot_positions(3, 1, n_peers, half, 256, s)
    ops = _neighbourhood_ops(np.zeros(n_peers, np.uint32), peer_pos, 16)
    pos = hotspot_positions(3, 2, n_msgs, half, 256, s)
    sender = stream(3, 3).below(n_peers, n_msgs)
    return Workload("C3", 16, ops, pos, np.zeros(n_msgs, np.uint32), sender, np.zeros(n_msgs, np.uint8), n_peers)


def _moves_to_ops(world, peers, old, new, s: int) -> np.ndarray:
    """AreaUnsubscribe for the cells of old + s*d that new + s*d no longer covers, then
    AreaSubscribe for the cells newly covered (positions, quantised by the table like the reference
    handlers do). Quantisation is per axis, so a peer's 27 cells are the product of three per-axis
    triples {cell(v - s), cell(v), cell(v + s)}: a cell is left iff one of its axis values is not in
    the new triple of that axis."""
    peers = np.asarray(peers, np.uint32)
    world = np.asarray(world, np.uint32)
    # only peers whose own cell changed can change their 27 cells
    ch = (cell_keys(old, s) != cell_keys(new, s)).any(1)
    if not ch.all():
        world, peers, old, new = world[ch], peers[ch], old[ch], new[ch]
    n = len(peers)
    if n == 0:
        return np.zeros(0, abi.OP_DTYPE)
    step = s * np.array([-1.0, 0.0, 1.0])
    d = (NEIGHBOURHOOD + 1).astype(np.int64)                          # (27, 3) axis indices
    keep_old = np.ones((n, 27), bool)
    keep_new = np.ones((n, 27), bool)
    for ax in range(3):
        to = cell_keys(old[:, ax, None] + step, s)                    # (n, 3)
        tn = cell_keys(new[:, ax, None] + step, s)
        in_new = (to[:, :, None] == tn[:, None, :]).any(2)            # old axis value still covered
        in_old = (tn[:, :, None] == to[:, None, :]).any(2)
        keep_old &= in_new[:, d[:, ax]]
        keep_new &= in_old[:, d[:, ax]]
    left, entered = ~keep_old, ~keep_new
    po = old[:, None, :] + s * NEIGHBOURHOOD[None, :, :]               # (n, 27, 3)
    pn = new[:, None, :] + s * NEIGHBOURHOOD[None, :, :]
    rw = np.repeat(world, 27).reshape(n, 27)
    rp = np.repeat(peers, 27).reshape(n, 27)
    un = abi.ops_array(rw[left], rp[left], np.full(int(left.sum()), abi.OP_UNSUBSCRIBE, np.uint8), pos=po[left])
    su = abi.ops_array(rw[entered], rp[entered], np.full(int(entered.sum()), abi.OP_SUBSCRIBE, np.uint8),
                       pos=pn[entered])
    return abi.concat_ops([un, su])


@dataclass
class ChurnWorld:
    """C4 state: peer worlds and positions, and the op / message stream of each tick."""
    world: np.ndarray     # (N,) u32 world of each peer
    pos: np.ndarray       # (N, 3) current positions
    half: float
    cube_size: int = 16
    tick_no: int = 0

    @property
    def n_peers(self) -> int:
        return len(self.world)

    def initial_ops(self) -> np.ndarray:
        return _neighbourhood_ops(self.world, self.pos, self.cube_size)

    def step(self, move_frac: float = 0.05):
        """One tick: (ops, msg_pos, msg_world, msg_sender, msg_repl). 5% of the peers move by
        N(0,16)^3 (clamped to the box); messages are one per peer at its new position, ExceptSelf."""
        self.tick_no += 1
        g = stream(4, 1000 + self.tick_no)
        N = self.n_peers
        moved = np.flatnonzero(g.uniform(0.0, 1.0, N) < move_frac).astype(np.uint32)
        old = self.pos[moved].copy()
        new = old + np.stack([g.normal(len(moved)) for _ in range(3)], 1) * 16.0
        new = np.clip(new, -self.half, np.nextafter(self.half, -np.inf))
        self.pos[moved] = new
        ops = _moves_to_ops(self.world[moved], moved, old, new, self.cube_size)
        return ops, self.pos.copy(), self.world.copy(), np.arange(N, dtype=np.uint32), np.zeros(N, np.uint8)


def config_c4(scale: float = 1.0, worlds=None) -> ChurnWorld:
    """C4: 64 worlds x 50k peers; `worlds` = the subset one GPU owns (e.g. range(r, 64, G))."""
    per = max(1, int(round(50_000 * scale)))
    half = 256.0 * (scale ** (1.0 / 3.0))
    ws = np.array(list(worlds) if worlds is not None else list(range(64)), dtype=np.uint32)
    world = np.repeat(ws, per)
    pos = stream(4, 1).uniform(-half, half, 3 * len(world)).reshape(-1, 3)
    return ChurnWorld(world, pos, half)


@dataclass
class MovingEntities:
    """C5 state: N entities; each tick every entity moves by its velocity (reflecting at the box),
    re-subscribes its 3x3x3 (ops = the cell difference) and sends one message at its position."""
    pos: np.ndarray
    vel: np.ndarray
    half: float
    cube_size: int = 16
    radius: float = 16.0
    tick_no: int = 0

    @property
    def n(self) -> int:
        return len(self.pos)

    def initial_ops(self) -> np.ndarray:
        return _neighbourhood_ops(np.zeros(self.n, np.uint32), self.pos, self.cube_size)

    def messages(self):
        n = self.n
        return self.pos.copy(), np.zeros(n, np.uint32), np.arange(n, dtype=np.uint32), np.zeros(n, np.uint8)

    def step(self) -> np.ndarray:
        """Move every entity one tick; returns the subscription ops of the move."""
        self.tick_no += 1
        old = self.pos.copy()
        new = old + self.vel
        out = np.abs(new) >= self.half  # bounce off the box: reverse, stay put this tick
        self.vel = np.where(out, -self.vel, self.vel)
        new = np.where(out, old, new)
        self.pos = new
        return _moves_to_ops(np.zeros(self.n, np.uint32), np.arange(self.n, dtype=np.uint32), old, new,
                             self.cube_size)


def config_c5(scale: float = 1.0) -> MovingEntities:
    n = max(1, int(round(1_000_000 * scale)))
    half = 1024.0 * (scale ** (1.0 / 3.0))
    pos = stream(5, 1).uniform(-half, half, 3 * n).reshape(n, 3)
    vel = stream(5, 2).uniform(-4.0, 4.0, 3 * n).reshape(n, 3)
    return MovingEntities(pos, vel, half)
