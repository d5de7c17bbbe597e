#!/usr/bin/env python3
"""Headline benchmark: routed message->peer pairs per second per tick, % of the HBM roofline.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

--gpus N > 1 without a launcher (no WORLD_SIZE in the environment): this process makes no GPU call,
starts N ranks of itself (RANK / LOCAL_RANK / WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free port), passes
rank 0's line through and exits with the first non-zero rank status. Under a launcher, --gpus must
equal WORLD_SIZE (exit status 2 otherwise). Exit status 3: the headline line was printed but the
second multi-GPU form (extra.cube_hash / extra.replicated_table) failed or hung.

Headline workload: SURVEY.md §8(d) C3, the configuration north_star's target is quoted on — 1M peers
each subscribed to a 3x3x3 neighbourhood (27M subscriptions), 10M LocalMessages per tick, 90% from
256 Zipf-weighted Gaussian hotspots, cube_size 16, ExceptSelf, synthetic (splitmix64).
  N = 1   the whole configuration on one GPU: every step is one full tick of the hot path on
          HBM-resident inputs (quantise -> probe -> filter -> CSR offsets + (msg, peer) pairs), with
          the C2 line (BASELINE.json configs[1]: 100k peers, 1M messages) nested under extra.c2.
  N > 1   strong scaling: every rank ingests M/N of the tick's messages. Headline: the replicated
          table (every GPU holds the whole ~10 GB table and routes its slice with the single-GPU
          tick, no exchange; DESIGN.md §6 says why); beside it, extra.cube_hash: the cube-hash
          sharded tick over RCCL (20-byte slots to the owners, row references + cube-list pools
          back; wq_sharded_route_tick_device), and under it pairs_on_owner: the owner form
          (wq_sharded_route_owner_slots_async: slots to the owners, the pairs left there). --shard
          cube or --shard owner makes that form the headline (extra: the replicated table).
The table is built once before timing. Every timed loop is checked afterwards through the
routers' sticky health words (wq_route_health): no tick may have given up or overflowed.
Other configs: --config c1 | c2 | c4 | c5 (bench_configs.py); --config c2 --shard cube = one world
of N x the C2 volume over the same sharded tick (weak scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md (HBM3E peak BW)
METRIC = "routed msg→peer pairs/sec per tick at 1/2/4/8 GPUs; % HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of the run; default WORLD_SIZE under a launcher, else 1")
    ap.add_argument("--config", choices=["c1", "c2", "c3", "c4", "c5"], default=None,
                    help="default: the headline, C3 (north_star's 1M peers / 10M messages per tick) with the C2 "
                         "line nested under extra.c2 at N = 1; c1..c5 = one SURVEY.md §8(d) config alone")
    ap.add_argument("--no-extra", action="store_true", help="headline only (skip the nested C2 line)")
    ap.add_argument("--c2-world", type=int, default=0, help="C2 in this world id (>= 1023: the wide-key path)")
    ap.add_argument("--c2-shift", type=float, default=0.0,
                    help="C2 translated by this much on every axis (e.g. 2.5e7: Minecraft-scale coordinates)")
    ap.add_argument("--steps", type=int, default=None, help="timed ticks (default c3/c5 10, c4 20, c1/c2 50)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed ticks (default c1/c2 200, c3 20: ~12-30 ms, so the clocks have ramped; c4/c5 2)")
    ap.add_argument("--scale", type=float, default=1.0, help="shrink C2 (tests only; 1.0 = the headline)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bound on the CPU baseline's routing work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard", choices=["world", "cube", "replicate", "owner"], default="world",
                    help="multi-GPU partitioning (see module docstring); C3: replicate (the default at N > 1), "
                         "cube (pairs returned to the ingesting GPU) or owner (pairs left on the owning GPU) as "
                         "the headline form")
    ap.add_argument("--pmc-file", default=os.path.join(ROOT, "profiles", "r02_pmc_route.json"),
                    help="rocprofv3 --pmc summary of the C2 tick (roofline.traffic)")
    a = ap.parse_args()
    a.headline = a.config is None
    if a.headline:
        a.config = "c3"
    _default_steps(a)
    return a


def _default_steps(a):
    if a.steps is None:
        a.steps = {"c1": 50, "c2": 50, "c3": 10, "c4": 20, "c5": 10}[a.config]
    if a.warmup is None:
        # untimed ticks long enough for the GPU clocks to ramp after the host-side table build
        # (measured: C2 61.3 us after 10 warm-up ticks, 60.0 us after 500; C3 1.423 / 1.412 ms
        # after 2 / 30)
        a.warmup = {"c1": 200, "c2": 200, "c3": 20}.get(a.config, 2)


def algorithmic_bytes(M: int, F: int, P: int) -> int:
    """B = M*(24 pos + 4 world + 4 sender + 1 repl) + M*32 bucket record
    + F*4 candidate ids + P*8 (u32 msg, u32 peer) + (M+1)*4 CSR offsets."""
    return 69 * M + 4 * F + 8 * P + 4


def timed_ticks(tick, steps: int, stream, dev, world_size: int, routers=()) -> float:
    """The timed region of every bench line: barrier + synchronize, `steps` calls of tick() between
    two HIP events on the launch stream, synchronize + barrier; milliseconds. Afterwards every
    router's sticky health words (wq_route_health) must be clean — the run's counters were never
    read, so this is what proves no timed tick gave up a spin or overflowed its capacity."""
    import torch
    import torch.distributed as dist
    for r in routers:
        r.route_health()  # clear whatever the untimed ticks left
    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(steps):
        tick()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world_size > 1:
        dist.barrier()
    for r in routers:
        r.check_health()
    return ev0.elapsed_time(ev1)


def roofline(B: int, tick_s: float, kernel: str, traffic=None, event_us=None) -> dict:
    """roofline for a tick moving B algorithmic bytes in tick_s seconds: the
    time is the timed region's ms_per_step (every launch of the tick, back to back), never the
    event-bracketed per-launch time, which carries event overhead (event_us, for reference)."""
    achieved = B / tick_s / 1e9
    out = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kernel, "tick_us": tick_s * 1e6,
           "algorithmic_bytes": B}
    if event_us is not None:
        out["kernel_event_us"] = event_us
    return out


def shard_workload(rank: int, scale: float = 1.0, world: int = 0, shift: float = 0.0):
    """World-sharded weak scaling: rank r owns world r (its own peers and its own tick of
    messages); no message crosses ranks, so there is no exchange step.
    world / shift move the C2 box to another world id / far from the origin (same fan-out)."""
    from worldql_server_amd import synth
    w = synth.config_c2(scale=scale, world_offset=world + rank)
    if shift:
        w.pos += shift
        w.ops["pos"] += shift
    return w


def cube_workload(rank: int, world_size: int, scale: float = 1.0):
    """Cube-hash weak scaling: one world of G x the C2 volume and peers; every rank generates the
    same subscription stream and ingests its own 1M-message slice of the tick."""
    from worldql_server_amd import synth
    G = world_size
    n_peers = max(1, int(round(100_000 * scale * G)))
    n_msgs = max(1, int(round(1_000_000 * scale))) * G
    half = 512.0 * ((scale * G) ** (1.0 / 3.0))
    w = synth.uniform_box(2, n_peers, n_msgs, half, neighbourhood=True)
    lo, hi = rank * n_msgs // G, (rank + 1) * n_msgs // G
    return w, lo, hi


def sysfs_clocks() -> dict:
    """The current DPM levels the amdgpu driver reports (pp_dpm_sclk / pp_dpm_mclk, the line marked
    '*') of every card the box exposes; best effort (empty when sysfs is not readable)."""
    import glob
    out = {}
    for kind in ("sclk", "mclk", "fclk"):
        vals = set()
        for f in sorted(glob.glob(f"/sys/class/drm/card*/device/pp_dpm_{kind}")):
            try:
                with open(f) as fh:
                    for ln in fh:
                        if ln.rstrip().endswith("*"):
                            vals.add(ln.split(":", 1)[-1].strip().rstrip("*").strip())
            except OSError:
                pass
        if vals:
            out[f"dpm_{kind}"] = sorted(vals)
    return out


def allreduce(vals, op: str, dev, world_size: int) -> list:
    """All-reduce a few float64 values over the ranks ("max" or "sum"). RCCL takes device tensors;
    gloo (the one-GPU rehearsal) takes host tensors — a device tensor handed to gloo is read by its
    own copy, unordered with the stream that wrote it (how an N = 2 rehearsal once summed bytes to 0)."""
    import torch
    import torch.distributed as dist
    vals = [float(v) for v in vals]
    if world_size == 1:
        return vals
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor(vals, dtype=torch.float64, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return t.cpu().tolist()


def reduce_over_ranks(t_ms: float, pairs: int, dev, world_size: int):
    """(max over ranks of the timed region, sum over ranks of pairs per tick)."""
    (t,) = allreduce([t_ms], "max", dev, world_size)
    (p,) = allreduce([pairs], "sum", dev, world_size)
    return t, p


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """--gpus N > 1 without a launcher: N ranks of this script, one per GPU, started from a process
    that has made no GPU call (it never imports torch). Returns the exit status: 0, or the first
    non-zero rank status (the other ranks are then stopped)."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with status {rc}; stopping the others",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return status


def _oracle_router(w):
    """The C restatement with the workload's table, and a chunk router over wqo_route (no sorting
    of recipients: the reference's AHashSet order is unordered too)."""
    import ctypes
    from oracle import oracle as orc
    o = orc.COracle(w.cube_size)
    t0 = time.perf_counter()
    o.apply_ops(w.ops)
    build_s = time.perf_counter() - t0
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)

    def run(lo_hi):
        lo, hi = lo_hi
        n = hi - lo
        offs = np.empty(n + 1, np.uint32)
        cap = 64 * n + 64
        peers = np.empty(cap, np.uint32)
        pos, wo = np.ascontiguousarray(w.pos[lo:hi]), np.ascontiguousarray(w.world[lo:hi])
        se, rp = np.ascontiguousarray(w.sender[lo:hi]), np.ascontiguousarray(w.repl[lo:hi])
        F = ctypes.c_uint64()
        P = o.lib.wqo_route(o.h, vp(pos), None, vp(wo), vp(se), vp(rp), n, vp(offs), vp(peers), cap, ctypes.byref(F))
        assert P <= cap
        return P

    return o, run, build_s


def cpu_baseline(w, seconds: float) -> dict:
    """The C restatement (oracle/wq_oracle.c: hash map world -> cube -> peer set, one message at
    a time), single thread, on a bounded sample of the same tick (whole chunks of 100k messages
    until `seconds` of routing have run)."""
    o, run, build_s = _oracle_router(w)
    M = len(w.world)
    chunk = min(M, 100_000)
    pairs, msgs, t_route, start = 0, 0, 0.0, 0
    while t_route < seconds and msgs < M:
        t0 = time.perf_counter()
        pairs += run((start, min(M, start + chunk)))
        t_route += time.perf_counter() - t0
        msgs += min(M, start + chunk) - start
        start += chunk
    o.close()
    return {"value": pairs / t_route, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"{msgs} of the tick's {M} messages ({pairs} pairs) routed in {t_route:.2f} s by "
                      f"oracle/wq_oracle.c on 1 host thread; table of {len(w.ops)} subscriptions built "
                      f"in {build_s:.2f} s (not timed)"}


def cpu_baseline_mt(w, threads: int) -> dict:
    """SURVEY.md §8(d) cpu_ref_mt: the same C restatement, read-only lookups in parallel over
    message chunks on `threads` host threads (ctypes releases the GIL during each call); the
    whole tick is routed."""
    from concurrent.futures import ThreadPoolExecutor
    o, run, _ = _oracle_router(w)
    M = len(w.world)
    bounds = np.linspace(0, M, 4 * threads + 1).astype(np.int64)
    chunks = [(int(bounds[i]), int(bounds[i + 1])) for i in range(len(bounds) - 1)]
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, chunks[:threads]))  # warm-up
        t0 = time.perf_counter()
        pairs = sum(ex.map(run, chunks))
        t = time.perf_counter() - t0
    o.close()
    return {"value": pairs / t, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"the whole tick ({M} messages, {pairs} pairs) in {t:.3f} s by oracle/wq_oracle.c "
                      f"on {threads} host threads (read-only lookups, {len(chunks)} chunks)"}


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ:
        if a.gpus is not None and a.gpus > 1:
            sys.exit(launch_ranks(a.gpus))
    elif a.gpus is not None and a.gpus != int(os.environ["WORLD_SIZE"]):
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}", file=sys.stderr, flush=True)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # WQ_BENCH_ONE_GPU=1: a rehearsal of the N > 1 control flow with every rank on cuda:0 over gloo
    # (RCCL refuses two ranks on one GPU); its timings mean nothing
    rehearse = os.environ.get("WQ_BENCH_ONE_GPU") == "1"
    if rehearse:
        local_rank = 0
    torch.cuda.set_device(local_rank)  # before the process group: RCCL's barrier uses the current device
    if world_size > 1:
        dist.init_process_group("gloo" if rehearse else "nccl", init_method="env://")
    dev = torch.device("cuda", local_rank)

    if a.config != "c2":
        import bench_configs
        out = bench_configs.run(a, rank, world_size, local_rank, dev)
    elif a.shard == "cube":
        out = run_cube(a, rank, world_size, local_rank, dev)
    else:
        out = run_c2(a, rank, world_size, local_rank, dev)
    if a.headline and world_size == 1 and not a.no_extra:
        # the C2 line (BASELINE.json configs[1]) beside the C3 headline, with its own steps
        import copy
        a2 = copy.copy(a)
        a2.config, a2.steps, a2.warmup, a2.headline = "c2", None, None, False
        _default_steps(a2)
        out["extra"] = {"c2": run_c2(a2, rank, world_size, local_rank, dev)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world_size > 1:
        dist.destroy_process_group()


def run_c2(a, rank, world_size, local_rank, dev) -> dict:
    """C2 (BASELINE.json configs[1]): one world per GPU, 100k peers x 27 cubes, 1M messages."""
    import torch
    from worldql_server_amd import abi
    from worldql_server_amd.router import Router

    w = shard_workload(rank, a.scale, a.c2_world, a.c2_shift)
    M = len(w.world)
    r = Router(w.cube_size, local_rank)
    stream = torch.cuda.Stream(device=dev)  # a real stream object: its handle is never the NULL stream
    r.set_stream(stream.cuda_stream)
    t0 = time.perf_counter()
    r.apply_ops(w.ops)
    build_s = time.perf_counter() - t0
    st = r.stats()

    pos = torch.from_numpy(w.pos).to(dev)
    world = torch.from_numpy(w.world.view(np.int32)).to(dev)
    sender = torch.from_numpy(w.sender.view(np.int32)).to(dev)
    repl = torch.from_numpy(w.repl).to(dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)  # uploads ran on the default stream

    def counters():
        torch.cuda.synchronize(dev)
        return cnt.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]

    # sizing tick (capacity 0: counts only), then exact-size outputs
    r.route_device(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
                   0, 0, 0, cnt.data_ptr())
    P = int(counters()["n_pairs"])
    cap = P + 1024
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    args = (pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
            peers.data_ptr(), msgs.data_ptr(), cap)

    def tick(c=0):
        r.route_device(*args, c)

    for _ in range(a.warmup):
        tick()
    tick(cnt.data_ptr())
    c = counters()
    P, F = int(c["n_pairs"]), int(c["n_candidates"])
    assert c["overflow"] == 0 and c["error"] == 0, c

    t_ms = timed_ticks(tick, a.steps, stream, dev, world_size, [r])
    t_max_ms, pairs_all = reduce_over_ranks(t_ms, P, dev, world_size)

    # kernel-only time of the route launch: HIP events recorded on the launch stream around
    # every route kernel (wq_profile_enable), separate pass so the headline loop is untouched
    r.profile_enable(True)
    for _ in range(a.steps):
        tick()
    k_ms, launches = r.profile_read()
    r.profile_enable(False)
    k_avg_s = k_ms / launches / 1e3
    B = algorithmic_bytes(M, F, P)
    traffic = None
    if os.path.exists(a.pmc_file):
        with open(a.pmc_file) as f:
            pmc = json.load(f)
        if pmc.get("messages_per_tick") == M and pmc.get("pairs_per_tick") == P:
            traffic = pmc.get("hbm_bytes_per_launch")

    out = {
        "metric": METRIC,
        "value": pairs_all * a.steps / (t_max_ms / 1e3),
        "unit": "pairs/s",
        "n_gpus": world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": t_max_ms / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (splitmix64, SURVEY.md §8(d) C2 generator)",
        "config": {
            "workload": "C2: 1 world/GPU, 100k peers x 3x3x3 cubes, 1M LocalMessages/tick, U[-512,512)^3, "
                        "cube_size 16, ExceptSelf" + ("" if a.scale == 1.0 else f" (scaled {a.scale})")
                        + (f", world id {a.c2_world}" if a.c2_world else "")
                        + (f", box translated by {a.c2_shift:g} per axis" if a.c2_shift else ""),
            "messages_per_tick": M, "peers": w.n_peers, "subscriptions": int(st["n_entries"]),
            "cubes": int(st["n_cubes"]), "pairs_per_tick": P, "candidates_per_tick": F,
            "parallelism": f"world-sharded x{world_size}", "table_build_s": round(build_s, 3),
        },
        "roofline": roofline(B, t_max_ms / a.steps / 1e3, "route tick (single launch: tick_kernel)", traffic,
                             k_avg_s * 1e6),
    }
    if rank == 0 and world_size == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(w, a.cpu_seconds)
        threads = min(16, os.cpu_count() or 1)
        if threads > 1:
            out["cpu_baseline_mt"] = cpu_baseline_mt(w, threads)
    r.close()
    return out


def run_cube(a, rank, world_size, local_rank, dev):
    """--shard cube: one world of N x the C2 volume sharded by cube hash through the C ABI's
    sharded tick (wq_sharded_route_tick_device over RCCL), timed end to end, exchanges included."""
    import torch
    import bench_configs
    from worldql_server_amd.router import Router

    w, lo, hi = cube_workload(rank, world_size, a.scale)
    M = hi - lo
    stream = torch.cuda.Stream(device=dev)
    r = Router(w.cube_size, local_rank)
    r.set_stream(stream.cuda_stream)
    if world_size > 1:
        bench_configs.attach_rccl(r, rank, world_size)
    t0 = time.perf_counter()
    r.sharded_apply_ops(w.ops)
    build_s = time.perf_counter() - t0
    st = r.stats()
    pos = torch.from_numpy(w.pos[lo:hi]).to(dev)
    world = torch.from_numpy(w.world[lo:hi].view(np.int32)).to(dev)
    sender = torch.from_numpy(w.sender[lo:hi].view(np.int32)).to(dev)
    repl = torch.from_numpy(w.repl[lo:hi]).to(dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = 24 * M + 1024
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    state = {"P": 0}

    def tick():
        rc, P = r.sharded_route_device(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M,
                                       offs.data_ptr(), peers.data_ptr(), msgs.data_ptr(), cap)
        assert rc == 0, (rc, P)
        state["P"] = P

    for _ in range(max(a.warmup, 1)):
        tick()
    t_ms = timed_ticks(tick, a.steps, stream, dev, world_size, [r])
    t_max_ms, pairs_all = reduce_over_ranks(t_ms, state["P"], dev, world_size)
    out = {
        "metric": METRIC,
        "value": pairs_all * a.steps / (t_max_ms / 1e3),
        "unit": "pairs/s",
        "n_gpus": world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": t_max_ms / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (splitmix64, SURVEY.md §8(d) C2 generator, volume and peers x n_gpus)",
        "config": {
            "workload": f"C2 x{world_size}: 1 world, {w.n_peers} peers x 3x3x3 cubes, 1M LocalMessages/GPU/tick, "
                        "cube_size 16, ExceptSelf" + ("" if a.scale == 1.0 else f" (scaled {a.scale})"),
            "messages_per_tick": M * world_size, "messages_per_gpu": M, "peers": w.n_peers,
            "subscriptions_this_shard": int(st["n_entries"]), "pairs_per_tick": int(pairs_all),
            "parallelism": f"cube-hash x{world_size}" + (" (RCCL all-to-all)" if world_size > 1 else ""),
            "table_build_s": round(build_s, 3),
        },
        "roofline": roofline(algorithmic_bytes(M, int(pairs_all) // world_size, int(pairs_all) // world_size),
                             t_max_ms / a.steps / 1e3, "whole sharded tick per GPU (shard + exchanges + owner route "
                             "+ unshard)"),
    }
    if rank == 0 and world_size == 1 and not a.no_cpu_baseline:
        w1 = shard_workload(0, a.scale)
        out["cpu_baseline"] = cpu_baseline(w1, a.cpu_seconds)
    r.close()
    return out


if __name__ == "__main__":
    main()
