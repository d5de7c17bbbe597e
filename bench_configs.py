"""bench.py --config c1 | c3 | c4 | c5: the SURVEY.md §8(d) configurations beside the headline.

Every mode prints one JSON line in bench.py's format (metric = routed pairs/s; value = all ranks'
pairs over the max-over-ranks time of the timed ticks). Inputs are generated and uploaded before
the timed region; a tick's timed work is everything the tick does on the GPU.

  c1  the reference's CPU-sized case (1k peers, 10k messages): GPU tick beside cpu_ref_1t and
      cpu_server_faithful_1t (the broadcast_to scan).
  c3  1M peers x 3x3x3 (S = 27M), 10M messages/tick, 90% from 256 Zipf-weighted Gaussian hotspots.
      N = 1: the whole configuration on one GPU. N > 1: strong scaling, every rank routes M/N
      messages — headline the replicated table (no exchange), beside it the cube-hash sharded tick
      over RCCL (extra.cube_hash; --shard cube makes it the headline).
  c4  8 worlds x 50k peers per GPU (weak scaling; 8 GPUs = the 64 worlds of C4, world-sharded, no
      message exchange). A tick = that tick's AreaUnsubscribe/AreaSubscribe churn (5% of peers move
      by N(0,16)^3) applied incrementally on the device (wq_apply_ops_device), then one message per
      peer at its new position (ExceptSelf).
  c5  1M entities moving U[-4,4)^3 per tick in U[-1024,1024)^3, 3x3x3 subscriptions, one message
      each; a tick = the subscription diff of the move (incremental), the new peer positions, and the
      route with the exact radius filter r = 16. N = 1: one GPU. N > 1: strong scaling by cube hash
      (the slot tick: owners return rows and pools, every rank holds all positions and filters).
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

import bench
from bench import HBM_PEAK_GBS, METRIC, algorithmic_bytes, reduce_over_ranks, roofline, timed_ticks

PMC_C3 = "r06_pmc_route_c3.json"  # rocprofv3 --pmc summary of the C3 tick on the round-6 build (dense headers,
                                   # aligned lists; tools/pmc_route.sh 10 --workload c3; x2 calibrated:
                                   # r04_fetch_calibration.json)


def run(a, rank, world_size, local_rank, dev):
    return {"c1": run_c1, "c3": run_c3, "c4": run_c4, "c5": run_c5}[a.config](a, rank, world_size, local_rank, dev)


def _line(a, world_size, value, ms_per_step, scaling, workload, config, roofline, data):
    return {"metric": METRIC, "value": value, "unit": "pairs/s", "n_gpus": world_size, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "f64", "data": data,
            "config": {"workload": workload, **config}, "roofline": roofline}


def _pmc_traffic(name: str, M: int, P: int):
    """HBM bytes per tick from a committed rocprofv3 --pmc summary (tools/pmc_route.sh +
    tools/pmc_summary.py) of the same workload, or None when there is none for this (M, P)."""
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    if d.get("messages_per_tick") != M or d.get("pairs_per_tick") != P:
        return None
    return d["hbm_bytes_per_launch"]


def _pmc_tick_traffic(name: str, scale: float):
    """HBM bytes per whole C4 / C5 tick from a committed tools/pmc_churn.sh summary (the bench's own
    deterministic workload, averaged over its 12 profiled ticks), or None (other scales)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", name)
    if scale != 1.0 or not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)["hbm_bytes_per_tick"]


def _counters(cnt):
    from worldql_server_amd import abi
    return cnt.cpu().numpy().view(abi.COUNTERS_DTYPE)


# ---- C1 ---------------------------------------------------------------------------------------

def _cpu_c1(w, repeats: int):
    """C1 on 1 host thread, whole tick, by the C restatement: cpu_ref_1t (wqo_route) and
    cpu_server_faithful_1t (wqo_route_faithful: + PeerMap::broadcast_to's per-message recipient
    set and O(|PeerMap|) scan over all 1,000 connected peers, peer_map.rs:151-163)."""
    import ctypes
    o, run, build_s = bench._oracle_router(w)
    M = len(w.world)
    vp = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    run((0, M))
    t0 = time.perf_counter()
    for _ in range(repeats):
        P = run((0, M))
    t_ref = (time.perf_counter() - t0) / repeats
    connected = np.arange(w.n_peers, dtype=np.uint32)  # every peer connected, map order = id order
    offs = np.empty(M + 1, np.uint32)
    peers = np.empty(64 * M + 64, np.uint32)
    pos, wo, se, rp = (np.ascontiguousarray(x) for x in (w.pos, w.world, w.sender, w.repl))
    f = o.lib.wqo_route_faithful
    f.restype = ctypes.c_size_t
    f.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_size_t]
    t0 = time.perf_counter()
    for _ in range(repeats):
        P2 = f(o.h, vp(pos), vp(wo), vp(se), vp(rp), M, vp(connected), len(connected), vp(offs), vp(peers),
               len(peers))
    t_faith = (time.perf_counter() - t0) / repeats
    o.close()
    assert P2 == P, (P, P2)
    samp = f"the whole C1 tick ({M} messages, {P} pairs), mean of {repeats} runs, oracle/wq_oracle.c, 1 host thread"
    return ({"value": P / t_ref, "unit": "pairs/s", "cores": 1, "kind": "port", "sample": "cpu_ref_1t: " + samp},
            {"value": P / t_faith, "unit": "pairs/s", "cores": 1, "kind": "port",
             "sample": "cpu_server_faithful_1t (broadcast_to set + O(|PeerMap|) scan per message): " + samp})


def run_c1(a, rank, world_size, local_rank, dev):
    """BASELINE.json configs[0]: 1 world, 1k peers x 1 cube, 10k messages in U[-64,64)^3 — the
    reference's CPU-sized case. One GPU (world_size > 1 runs a replica per rank, weak)."""
    import torch
    from worldql_server_amd import synth
    from worldql_server_amd.router import Router
    w = synth.config_c1()
    M = len(w.world)
    r = Router(w.cube_size, local_rank)
    stream = torch.cuda.Stream(device=dev)
    r.set_stream(stream.cuda_stream)
    r.apply_ops(w.ops)
    pos = torch.from_numpy(w.pos).to(dev)
    world = torch.from_numpy(w.world.view(np.int32)).to(dev)
    sender = torch.from_numpy(w.sender.view(np.int32)).to(dev)
    repl = torch.from_numpy(w.repl).to(dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    r.route_device(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
                   0, 0, 0, cnt.data_ptr())
    torch.cuda.synchronize(dev)
    P = int(_counters(cnt)[0]["n_pairs"])
    cap = P + 1024
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    args = (pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
            peers.data_ptr(), 0, cap)
    for _ in range(a.warmup):
        r.route_device(*args, 0)
    r.route_device(*args, cnt.data_ptr())
    torch.cuda.synchronize(dev)
    c = _counters(cnt)[0]
    F = int(c["n_candidates"])
    assert c["overflow"] == 0 and c["error"] == 0, c
    t_ms = timed_ticks(lambda: r.route_device(*args, 0), a.steps, stream, dev, world_size, [r])
    t_max_ms, pairs_all = reduce_over_ranks(t_ms, P, dev, world_size)
    r.profile_enable(True)
    for _ in range(a.steps):
        r.route_device(*args, 0)
    k_ms, launches = r.profile_read()
    r.profile_enable(False)
    k_s = k_ms / launches / 1e3
    B = algorithmic_bytes(M, F, P)
    out = _line(a, world_size, pairs_all * a.steps / (t_max_ms / 1e3), t_max_ms / a.steps, "weak",
                "C1: 1 world, 1k peers x 1 cube, 10k LocalMessages/tick, U[-64,64)^3, cube_size 16, ExceptSelf "
                "(BASELINE.json configs[0], the reference's CPU case; launch-latency bound on a GPU)",
                {"messages_per_tick": M, "peers": w.n_peers, "pairs_per_tick": P, "candidates_per_tick": F,
                 "parallelism": f"replicas x{world_size}"},
                roofline(B, t_max_ms / a.steps / 1e3, "route tick (single launch)", None, k_s * 1e6),
                "synthetic (splitmix64, SURVEY.md §8(d) C1 generator)")
    if rank == 0 and world_size == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"], out["cpu_baseline_faithful"] = _cpu_c1(w, 20)
    r.close()
    return out


# ---- C3 ---------------------------------------------------------------------------------------

def run_c3(a, rank, world_size, local_rank, dev):
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Router

    t0 = time.perf_counter()
    w = synth_ext.config_c3(scale=a.scale)
    gen_s = time.perf_counter() - t0
    if world_size > 1 or a.shard in ("cube", "replicate", "owner"):
        # N > 1: both multi-GPU forms, the replicated table as the headline unless
        # --shard cube; --shard cube / replicate at N = 1: that form alone on one rank
        return _run_c3_multi(a, w, rank, world_size, local_rank, dev, gen_s)
    M = len(w.world)
    r = Router(w.cube_size, local_rank)
    stream = torch.cuda.Stream(device=dev)
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
    torch.cuda.synchronize(dev)
    r.route_device(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
                   0, 0, 0, cnt.data_ptr())
    torch.cuda.synchronize(dev)
    P = int(_counters(cnt)["n_pairs"][0])
    r.set_fanout_hint(P / M)  # a server passes its previous tick's P / M; C3's ~42 picks count/scan/emit
    cap = P + 1024
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    args = (pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
            peers.data_ptr(), msgs.data_ptr(), cap)
    for _ in range(a.warmup):
        r.route_device(*args, 0)
    r.route_device(*args, cnt.data_ptr())
    torch.cuda.synchronize(dev)
    c = _counters(cnt)[0]
    P, F = int(c["n_pairs"]), int(c["n_candidates"])
    assert c["overflow"] == 0 and c["error"] == 0, c
    t_ms = timed_ticks(lambda: r.route_device(*args, 0), a.steps, stream, dev, 1, [r])
    # the GPU's shader clock right after the timed region (the box-to-box spread of the headline is
    # partly clock: VERDICT r5 Weak #5), then one event-bracketed launch per tick with events between
    # its kernels, so the line says which kernel moved
    sclk_mhz = r.probe_sclk()
    r.profile_enable(True)
    for _ in range(a.steps):
        r.route_device(*args, 0)
    k_ms, launches, ph_ms, n_ph = r.profile_read_phases()
    r.profile_enable(False)
    k_avg_s = k_ms / launches / 1e3
    B = algorithmic_bytes(M, F, P)
    kernel = ("route tick (count / tile_scan / emit launches, wq_set_fanout_hint)" if P / M >= 16
              else "route tick (single launch: tick_kernel)")
    out = _line(a, 1, P * a.steps / (t_ms / 1e3), t_ms / a.steps, "strong",
                "C3: 1M peers x 3x3x3, 10M LocalMessages/tick, 256 Zipf(1) Gaussian hotspots (sigma 128) + 10% "
                "uniform in U[-4096,4096)^3, cube_size 16, ExceptSelf, whole configuration on one GPU"
                + ("" if a.scale == 1.0 else f" (scaled {a.scale})"),
                {"messages_per_tick": M, "peers": w.n_peers, "subscriptions": int(st["n_entries"]),
                 "cubes": int(st["n_cubes"]), "pairs_per_tick": P, "candidates_per_tick": F,
                 "parallelism": "1 GPU", "table_build_s": round(build_s, 3), "generate_s": round(gen_s, 1)},
                roofline(B, t_ms / a.steps / 1e3, kernel, _pmc_traffic(PMC_C3, M, P), k_avg_s * 1e6),
                "synthetic (splitmix64, SURVEY.md §8(d) C3 generator)")
    if n_ph:
        us = [x / n_ph * 1e3 for x in ph_ms]
        # per kernel: its own §8(d) share — count 69M (inputs + bucket record), emit 4F + 8P + 4(M+1)
        out["roofline"]["kernel_phases_us"] = {"count": round(us[0], 1), "tile_scan": round(us[1], 1),
                                               "emit": round(us[2], 1)}
        out["roofline"]["kernel_phase_frac"] = {
            "count": 69 * M / (us[0] * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "emit": (4 * F + 8 * P + 4 * (M + 1)) / (us[2] * 1e-6) / 1e9 / HBM_PEAK_GBS}
    out["clocks"] = {"sclk_mhz_after_timed_region": round(sclk_mhz, 1), **bench.sysfs_clocks()}
    # SURVEY.md §8(b)'s output contract proper: CSR offsets[M+1] + peers[P], msgs = NULL (no per-pair
    # message index: the caller hands message m its slice peers[offsets[m] .. offsets[m+1]) as
    # broadcast_to does). Same tick, same inputs; its peers are checked equal to the full form's.
    ref_offs, ref_peers = offs.clone(), peers[:P].clone()
    args_csr = args[:7] + (0, cap)
    t2_ms = timed_ticks(lambda: r.route_device(*args_csr, 0), a.steps, stream, dev, 1, [r])
    torch.cuda.synchronize(dev)
    assert torch.equal(offs, ref_offs) and torch.equal(peers[:P], ref_peers), "CSR-only tick differs"
    del ref_offs, ref_peers
    B2 = B - 4 * P  # no msgs[P] written
    out["csr_only"] = {"value": P * a.steps / (t2_ms / 1e3), "unit": "pairs/s", "ms_per_step": t2_ms / a.steps,
                       "algorithmic_bytes": B2, "frac": B2 / (t2_ms / a.steps / 1e3) / 8e12,
                       "note": "the same C3 tick with msgs = NULL: offsets + peers only (SURVEY.md §8(b) output); "
                               "algorithmic bytes 69M + 4F + 4P + 4; peers checked equal to the full form's"}
    if not a.no_cpu_baseline:
        out["cpu_baseline"] = _cpu_route_sample(w, a.cpu_seconds, "C3")
        threads = min(16, os.cpu_count() or 1)
        if threads > 1:  # SURVEY.md §8(d) cpu_ref_mt: the same restatement on the host's cores
            out["cpu_baseline_mt"] = bench.cpu_baseline_mt(w, threads)
    out["xgmi_model"] = _xgmi_model()
    r.close()
    return out


XGMI_G8 = "r03_c3_xgmi_g8.json"  # tools/shard_volume.py --G 8: full C3 as 8 hub shards on one GPU
XGMI_LINK_GBS = 64.0  # one xGMI link, one direction, sustained (MI355X_MICROARCH.md: ~153 GB/s per link both ways)


def _xgmi_model():
    """What an 8-GPU cube-hash tick of this workload moves between GPUs, per GPU — measured, not
    estimated: tools/shard_volume.py runs the sharded tick with G = 8 hub shards on one GPU and
    reads wq_shard_last_bytes (the bytes each shard sends to / receives from the other seven).
    link_us: that volume spread over the 7 links of a GPU at XGMI_LINK_GBS each (a lower bound on
    the exchange time; the exchanges themselves are not overlapped with compute)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", XGMI_G8)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    out = {"n_gpus": d["G"], "source": "profiles/" + XGMI_G8 + " (tools/shard_volume.py)"}
    for form in ("slots", "expanded"):
        b = d[form]["sent_bytes_per_gpu_max"]
        out[form] = {"xgmi_bytes_per_gpu": b, "link_us": round(b / (7 * XGMI_LINK_GBS * 1e3), 1)}
    out["note"] = ("slots = the sharded tick's default (20-byte slots out, row references + one pool of cube lists "
                   "per destination back); expanded = 40-byte records out, expanded pairs back")
    return out


def _gloo_exchange(dist):
    """The caller's all-to-all (wq_shard_attach_exchange) over the bench's gloo group: device -> host,
    gloo, host -> device. Only for WQ_BENCH_ONE_GPU rehearsals (RCCL refuses two ranks on one GPU)."""
    import ctypes
    import torch
    hip = ctypes.CDLL("libamdhip64.so.7")  # the HIP runtime PyTorch already loaded
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]

    def fn(send, sb, recv, rb, stream):
        assert hip.hipStreamSynchronize(stream or None) == 0
        src = np.empty(max(sum(sb), 1), np.uint8)
        if sum(sb):
            assert hip.hipMemcpy(src.ctypes.data, send, sum(sb), 4) == 0
        dst = torch.empty(sum(rb), dtype=torch.uint8)
        dist.all_to_all_single(dst, torch.from_numpy(src[:sum(sb)]), list(rb), list(sb))
        if sum(rb):
            assert hip.hipMemcpy(recv, dst.numpy().ctypes.data, sum(rb), 4) == 0
    return fn


def attach_rccl(r, rank: int, world_size: int) -> None:
    """This rank's router becomes shard `rank` of world_size over its own RCCL communicator (the id
    travels over the bench's process group)."""
    import torch.distributed as dist
    from worldql_server_amd.router import rccl_unique_id
    if os.environ.get("WQ_BENCH_ONE_GPU") == "1" and world_size > 1:
        r.attach_exchange(world_size, rank, _gloo_exchange(dist))  # rehearsal: every rank on cuda:0
        return
    uid = [rccl_unique_id() if rank == 0 else None]
    if world_size > 1:
        dist.broadcast_object_list(uid, src=0)
    r.attach_rccl(world_size, rank, uid[0])


def _c3_slice(w, rank, world_size, dev):
    import torch
    M_all = len(w.world)
    lo, hi = rank * M_all // world_size, (rank + 1) * M_all // world_size
    t = (torch.from_numpy(w.pos[lo:hi]).to(dev), torch.from_numpy(w.world[lo:hi].view(np.int32)).to(dev),
         torch.from_numpy(w.sender[lo:hi].view(np.int32)).to(dev), torch.from_numpy(w.repl[lo:hi]).to(dev))
    torch.cuda.synchronize(dev)
    return lo, hi, t


def _c3_replicated(a, w, rank, world_size, local_rank, dev, stream, sl):
    """The replicated-table form (wq_router_create_multi_mode's WQ_MULTI_REPLICATE, one process per
    GPU): every rank holds the WHOLE table (C3: ~25 GB of 288 GB; every op applied on every GPU) and
    routes its own M/N messages with the single-GPU tick — no exchange at all."""
    import torch
    from worldql_server_amd.router import Router
    lo, hi, (pos, world, sender, repl) = sl
    M = hi - lo
    r = Router(w.cube_size, local_rank)
    r.set_stream(stream.cuda_stream)
    t0 = time.perf_counter()
    r.apply_ops(w.ops)
    build_s = time.perf_counter() - t0
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    r.route_device(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
                   0, 0, 0, cnt.data_ptr())
    torch.cuda.synchronize(dev)
    P = int(_counters(cnt)["n_pairs"][0])
    r.set_fanout_hint(P / max(M, 1))  # a server passes its previous tick's P / M
    cap = P + 1024
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    args = (pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
            peers.data_ptr(), msgs.data_ptr(), cap)
    for _ in range(max(a.warmup, 1)):
        r.route_device(*args, 0)
    r.route_device(*args, cnt.data_ptr())
    torch.cuda.synchronize(dev)
    c = _counters(cnt)[0]
    P, F = int(c["n_pairs"]), int(c["n_candidates"])
    assert c["overflow"] == 0 and c["error"] == 0, c
    t_ms = timed_ticks(lambda: r.route_device(*args, 0), a.steps, stream, dev, world_size, [r])
    r.close()
    (t_max_ms,) = bench.allreduce([t_ms], "max", dev, world_size)
    pairs_all, B_all = bench.allreduce([P, algorithmic_bytes(M, F, P)], "sum", dev, world_size)
    assert B_all > 0 and pairs_all >= 0, (B_all, pairs_all)
    del peers, msgs
    return {"t_max_ms": t_max_ms, "pairs_all": int(pairs_all), "B_all": int(B_all), "build_s": build_s,
            "P_rank": P, "M_rank": M}


def _c3_cube(a, w, rank, world_size, local_rank, dev, stream, sl, owner_form: bool):
    """The cube-hash form (wq_sharded_route_tick_device over RCCL): every rank holds the buckets it
    owns and ingests M/N messages; a tick sends the remote ones to their owners as 20-byte slots and
    gets back 12-byte row references + one pool of cube lists per owner, exchanges sized by budgets
    from the previous tick (one host read per tick, at its end)."""
    import torch
    from worldql_server_amd.router import Router
    lo, hi, (pos, world, sender, repl) = sl
    M = hi - lo
    r = Router(w.cube_size, local_rank)
    r.set_stream(stream.cuda_stream)
    attach_rccl(r, rank, world_size)
    t0 = time.perf_counter()
    r.sharded_apply_ops(w.ops)
    build_s = time.perf_counter() - t0
    st = r.stats()
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    r.set_fanout_hint(40.0)
    cap = 64 * M + 1024
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)

    def tick():
        # wq_sharded_route_tick_async: no end-of-tick read (the next tick's budgets come from the
        # tick before); P and the status bits land in cnt, every tick's bits in the sticky health
        # words that timed_ticks checks afterwards
        r.sharded_route_async(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M,
                              offs.data_ptr(), peers.data_ptr(), msgs.data_ptr(), cap, cnt.data_ptr())

    for _ in range(max(a.warmup, 2)):
        tick()
    t_ms = timed_ticks(tick, a.steps, stream, dev, world_size, [r])
    c = _counters(cnt)[0]
    assert c["error"] == 0 and c["overflow"] == 0, c
    exact, budgeted = r.shard_tick_stats()
    t_max_ms, pairs_all = reduce_over_ranks(t_ms, int(c["n_pairs"]), dev, world_size)
    # this form's own §8(d) bytes: every ingested message's 69 B, its candidates, its pairs with the
    # per-pair message index (the slot tick returns (message, peer) pairs to the ingesting GPU)
    (B_all,) = bench.allreduce([algorithmic_bytes(M, int(c["n_candidates"]), int(c["n_pairs"]))], "sum", dev,
                               world_size)
    sent, _ = r.shard_last_bytes()  # the last timed tick's bytes to the other GPUs (xGMI)
    sent_max, _ = reduce_over_ranks(float(sent), 0, dev, world_size)
    out = {"t_max_ms": t_max_ms, "pairs_all": int(pairs_all), "B_all": int(B_all), "build_s": build_s,
           "subscriptions_this_shard": int(st["n_entries"]), "xgmi_bytes_per_gpu": int(sent_max),
           "exact_ticks": exact, "budgeted_ticks": budgeted}
    if owner_form:
        # SURVEY.md §8(e) step 5's other option: the pairs left on the owner — wq_sharded_route_owner_slots_async,
        # budgeted 20-byte slots out and nothing back (one exchange per tick, no end-of-tick read)
        cnt_o = torch.zeros(24, dtype=torch.uint8, device=dev)

        def tick_owner():
            r.sharded_route_owner_slots_async(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M,
                                              cnt_o.data_ptr())
        for _ in range(max(a.warmup, 3)):
            tick_owner()
        e0, b0 = r.shard_tick_stats()
        t_ms = timed_ticks(tick_owner, a.steps, stream, dev, world_size, [r])
        e1, b1 = r.shard_tick_stats()
        co = _counters(cnt_o)[0]
        assert co["error"] == 0 and co["overflow"] == 0, co
        t2, pairs_own = reduce_over_ranks(t_ms, int(co["n_pairs"]), dev, world_size)
        assert pairs_own == pairs_all, (pairs_own, pairs_all)  # every pair routed exactly once
        # the owner form's OWN §8(d) bytes (VERDICT r5 Weak #3): 69 B per ingested message, its
        # candidates, its pairs written once (a CSR over the received slots, no per-pair message index)
        (B_own,) = bench.allreduce([69 * M + 4 * int(co["n_candidates"]) + 4 * int(co["n_pairs"]) + 4], "sum", dev,
                                   world_size)
        sent_o, _ = r.shard_last_bytes()
        sent_o_max, _ = reduce_over_ranks(float(sent_o), 0, dev, world_size)
        out["pairs_on_owner"] = {"value": pairs_own * a.steps / (t2 / 1e3), "unit": "pairs/s",
                                 "ms_per_step": t2 / a.steps, "xgmi_bytes_per_gpu": int(sent_o_max),
                                 "algorithmic_bytes_per_gpu": int(B_own) // world_size,
                                 "roofline_frac_per_gpu": B_own / world_size / (t2 / a.steps / 1e3) / 1e9 / HBM_PEAK_GBS,
                                 "exact_ticks_timed": e1 - e0, "budgeted_ticks_timed": b1 - b0,
                                 "note": "wq_sharded_route_owner_slots_async: the same tick's pairs left on the "
                                         "owning GPU (20-byte slots out, no return exchange, no end-of-tick read)"}
    r.close()
    del peers, msgs
    return out


def _c3_owner(a, w, rank, world_size, local_rank, dev, stream, sl):
    """The cube-hash owner form (wq_sharded_route_owner_slots_async over RCCL, SURVEY.md §8(e) step 5's
    first option): every rank holds the buckets it owns and ingests M/N messages; a tick sends every
    message to its owner as a 20-byte slot (budgeted sizes, one exchange, no end-of-tick read) and the
    owner routes it there, leaving the pairs on that GPU (a CSR over its received slots)."""
    import torch
    from worldql_server_amd.router import Router
    lo, hi, (pos, world, sender, repl) = sl
    M = hi - lo
    r = Router(w.cube_size, local_rank)
    r.set_stream(stream.cuda_stream)
    attach_rccl(r, rank, world_size)
    t0 = time.perf_counter()
    r.sharded_apply_ops(w.ops)
    build_s = time.perf_counter() - t0
    st = r.stats()
    r.set_fanout_hint(40.0)
    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)

    def tick():
        r.sharded_route_owner_slots_async(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M,
                                          cnt.data_ptr())
    for _ in range(max(a.warmup, 3)):
        tick()
    e0, b0 = r.shard_tick_stats()
    t_ms = timed_ticks(tick, a.steps, stream, dev, world_size, [r])
    e1, b1 = r.shard_tick_stats()
    c = _counters(cnt)[0]
    assert c["error"] == 0 and c["overflow"] == 0, c
    P, F = int(c["n_pairs"]), int(c["n_candidates"])
    sent, _ = r.shard_last_bytes()
    r.close()
    (t_max_ms,) = bench.allreduce([t_ms], "max", dev, world_size)
    # §8(d) bytes of the routing this GPU did: its ingested messages' 69 B, the candidates it read, and
    # its pairs written once (a CSR over its received slots: no per-pair message index)
    pairs_all, B_all = bench.allreduce([P, 69 * M + 4 * F + 4 * P + 4], "sum", dev, world_size)
    (sent_max,) = bench.allreduce([float(sent)], "max", dev, world_size)
    return {"t_max_ms": t_max_ms, "pairs_all": int(pairs_all), "B_all": int(B_all), "build_s": build_s,
            "subscriptions_this_shard": int(st["n_entries"]), "xgmi_bytes_per_gpu": int(sent_max),
            "exact_ticks_timed": e1 - e0, "budgeted_ticks_timed": b1 - b0}


def _run_c3_multi(a, w, rank, world_size, local_rank, dev, gen_s):
    """C3 over N GPUs, strong scaling (the 10M messages of a tick split over the ranks), both
    multi-GPU forms measured in the same run on the same slices:
      replicate   every GPU holds the whole table and routes its slice — the headline (DESIGN.md §6:
                  C3's table is ~25 GB of 288 GB, so the exchange the cube-hash form needs buys
                  nothing at this size; value = all ranks' pairs / the max-over-ranks time)
      cube        the cube-hash sharded tick over RCCL (the form for tables beyond one GPU's HBM),
                  under extra.cube_hash (--shard cube: the headline instead)
    Each timed region: barrier + synchronize, K ticks, synchronize + barrier, max over ranks."""
    import threading
    import torch
    head = a.shard if a.shard in ("cube", "owner") else "replicate"
    stream = torch.cuda.Stream(device=dev)
    sl = _c3_slice(w, rank, world_size, dev)
    M_all = len(w.world)
    M = sl[1] - sl[0]
    res = {}
    forms = [head] if (world_size == 1 or a.no_extra) else [head, "cube" if head == "replicate" else "replicate"]
    name = {"cube": "cube_hash", "replicate": "replicated_table", "owner": "owner_slots"}

    def line():
        h = res[head]
        t = h["t_max_ms"]
        B = (h["B_all"] if head == "owner" else res["replicate"]["B_all"] if "replicate" in res else
             algorithmic_bytes(M_all, h["pairs_all"], h["pairs_all"]))
        par = {"replicate": f"replicated table x{world_size} (every GPU holds all {len(w.ops)} subscriptions and routes "
                            f"its {M} of the {M_all} messages; no exchange)",
               "cube": f"cube-hash x{world_size} (wq_sharded_route_tick_device over RCCL: 20-byte slots out, row "
                       "references + per-destination cube-list pools back, budgeted exchanges)",
               "owner": f"cube-hash owner form x{world_size} (wq_sharded_route_owner_slots_async over RCCL: every "
                        "message to its owner as a 20-byte slot, one budgeted exchange, the pairs left on the "
                        "owning GPU)"}[head]
        cfg = {"messages_per_tick": M_all, "messages_per_gpu": M, "peers": w.n_peers,
               "pairs_per_tick": h["pairs_all"], "parallelism": par, "table_build_s": round(h["build_s"], 3),
               "generate_s": round(gen_s, 1)}
        if head in ("cube", "owner"):
            cfg.update({k: h[k] for k in h if k.startswith(("subscriptions", "xgmi", "exact", "budgeted"))})
        out = _line(a, world_size, h["pairs_all"] * a.steps / (t / 1e3), t / a.steps, "strong",
                    f"C3 over {world_size} GPU(s): 1M peers x 3x3x3, 10M LocalMessages/tick in total, "
                    "256 Zipf(1) Gaussian hotspots + 10% uniform, cube_size 16, ExceptSelf"
                    + ("" if a.scale == 1.0 else f" (scaled {a.scale})"), cfg,
                    roofline(B // world_size, t / a.steps / 1e3,
                             "whole tick per GPU; bytes = the tick's SURVEY §8(d) bytes / N" +
                             {"replicate": " (count / tile_scan / emit on each GPU's slice)",
                              "cube": " (own-cube count + slots + exchanges + owner count + pools + emit)",
                              "owner": " (pairs written once, no per-pair message index: grouping + exchange + "
                                       "owner count / tile_scan / emit)"}[head]),
                    "synthetic (splitmix64, SURVEY.md §8(d) C3 generator)")
        out["xgmi_model"] = _xgmi_model()
        extra = {}
        for f in forms[1:]:
            if f in res:
                x = res[f]
                e = {"value": x["pairs_all"] * a.steps / (x["t_max_ms"] / 1e3), "unit": "pairs/s",
                     "ms_per_step": x["t_max_ms"] / a.steps, "n_gpus": world_size, "scaling": "strong"}
                e.update({k: v for k, v in x.items() if k not in ("t_max_ms", "pairs_all", "B_all")})
                if "B_all" in x:  # each form on its OWN §8(d) bytes per GPU (link time included)
                    e["algorithmic_bytes_per_gpu"] = int(x["B_all"]) // world_size
                    e["roofline_frac_per_gpu"] = (x["B_all"] / world_size / (x["t_max_ms"] / a.steps / 1e3) / 1e9 /
                                                  HBM_PEAK_GBS)
                extra[name[f]] = e
            else:
                extra[name[f]] = {"error": "did not finish in time"}
        if extra:
            out["extra"] = extra
        return out

    for i, f in enumerate(forms):
        dog = None
        if i > 0:
            # the second form must not cost the headline: if it hangs (an RCCL collective that
            # never completes), rank 0 prints the headline line and every rank leaves
            def bail():
                if rank == 0:
                    print(json.dumps(line()), flush=True)
                print(f"rank {rank}: the {f} form did not finish in 120 s", file=sys.stderr, flush=True)
                os._exit(3)  # the headline stands, the run does not pass as clean
            dog = threading.Timer(120.0, bail)  # the cube form takes ~10 s when it works
            dog.daemon = True
            dog.start()
        try:
            if f == "replicate":
                res[f] = _c3_replicated(a, w, rank, world_size, local_rank, dev, stream, sl)
            elif f == "owner":
                res[f] = _c3_owner(a, w, rank, world_size, local_rank, dev, stream, sl)
            else:
                res[f] = _c3_cube(a, w, rank, world_size, local_rank, dev, stream, sl, owner_form=not a.no_extra)
        except Exception as e:  # noqa: BLE001
            if i == 0:
                raise
            # the second form failed on this rank: its peers may be inside a collective that will never
            # complete, so this rank reports (rank 0: the headline line, the error under extra) and
            # leaves; a peer still waiting leaves through its own watchdog
            print(f"rank {rank}: {f} form failed: {e!r}", file=sys.stderr, flush=True)
            if rank == 0:
                out = line()
                out.setdefault("extra", {})[name[f]] = {"error": repr(e)}
                print(json.dumps(out), flush=True)
            os._exit(3)  # the headline line stands; the failed form makes the run's status non-zero
        if dog:
            dog.cancel()
    for f in ("cube", "owner"):
        if "replicate" in res and f in res:
            assert res["replicate"]["pairs_all"] == res[f]["pairs_all"]  # the same pairs either way
    return line()


def _cpu_route_sample(w, seconds, name):
    """The C restatement on 1 host thread, routing a bounded prefix of the tick's messages."""
    o, run, build_s = bench._oracle_router(w)
    M = len(w.world)
    chunk = min(M, 50_000)
    pairs = msgs = 0
    t_route = 0.0
    start = 0
    while t_route < seconds and start < M:
        t0 = time.perf_counter()
        pairs += run((start, min(M, start + chunk)))
        t_route += time.perf_counter() - t0
        msgs += min(M, start + chunk) - start
        start += chunk
    o.close()
    return {"value": pairs / t_route, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"{name}: {msgs} of the tick's {M} messages ({pairs} pairs) routed in {t_route:.2f} s by "
                      f"oracle/wq_oracle.c on 1 host thread; table of {len(w.ops)} subscriptions built in "
                      f"{build_s:.1f} s (not timed)"}


# ---- C4 / C5: churn ticks ----------------------------------------------------------------------

def _ops_tensor(ops, dev):
    import torch
    raw = np.ascontiguousarray(ops).view(np.uint8)
    return torch.from_numpy(raw.copy()).to(dev)


def _churn_ticks(a, r, dev, stream, ticks, M, world_t, sender_t, repl_t, positions=False):
    """Runs the pregenerated ticks (ops, pos) through update + route; returns per-phase timings."""
    import torch
    ops_d = [_ops_tensor(t[0], dev) for t in ticks]
    n_ops = [len(t[0]) for t in ticks]
    pos_d = [torch.from_numpy(t[1]).to(dev) for t in ticks]
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = 80 * M + 1024
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = torch.zeros((len(ticks), 24), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)

    def one(i, c):
        r.apply_ops_device(ops_d[i].data_ptr(), n_ops[i])
        if positions:
            r.set_peer_positions_device(pos_d[i].data_ptr(), M)
        r.route_device(pos_d[i].data_ptr(), world_t.data_ptr(), sender_t.data_ptr(), repl_t.data_ptr(), M,
                       offs.data_ptr(), peers.data_ptr(), msgs.data_ptr(), cap, c)

    for i in range(a.warmup):
        one(i, cnt[i].data_ptr())
    torch.cuda.synchronize(dev)
    upd0, _ = r.update_counts()
    r.profile_enable(True)
    t0 = time.perf_counter()
    for i in range(a.warmup, a.warmup + a.steps):
        one(i, cnt[i].data_ptr())
    torch.cuda.synchronize(dev)
    t_ms = (time.perf_counter() - t0) * 1e3
    k_ms, launches = r.profile_read()
    r.profile_enable(False)
    upd1, fb = r.update_counts()
    c = _counters(cnt)[a.warmup:]
    assert (c["overflow"] == 0).all() and (c["error"] == 0).all()
    return {"t_ms": t_ms, "route_ms": k_ms, "launches": launches, "P": int(c["n_pairs"].sum()),
            "F": int(c["n_candidates"].sum()), "ops": int(sum(n_ops[a.warmup:])),
            "incremental": upd1 - upd0, "fallbacks": fb}


def run_c4(a, rank, world_size, local_rank, dev):
    import torch
    import torch.distributed as dist
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Router

    worlds = range(8 * rank, 8 * rank + 8)
    c4 = synth_ext.config_c4(scale=a.scale, worlds=worlds)
    t0 = time.perf_counter()
    init = c4.initial_ops()
    ticks = [c4.step()[:2] for _ in range(a.warmup + a.steps)]
    gen_s = time.perf_counter() - t0
    M = c4.n_peers
    stream = torch.cuda.Stream(device=dev)
    r = Router(16, local_rank)
    r.set_stream(stream.cuda_stream)
    if os.environ.get("WQ_BENCH_FANOUT_HINT"):  # tuning: the route shape a server's hint would pick
        r.set_fanout_hint(float(os.environ["WQ_BENCH_FANOUT_HINT"]))
    t0 = time.perf_counter()
    r.apply_ops(init)
    build_s = time.perf_counter() - t0
    S0 = r.stats()["n_entries"]
    world_t = torch.from_numpy(c4.world.view(np.int32)).to(dev)
    sender_t = torch.from_numpy(np.arange(M, dtype=np.int32)).to(dev)
    repl_t = torch.zeros(M, dtype=torch.uint8, device=dev)
    if world_size > 1:
        dist.barrier()
    res = _churn_ticks(a, r, dev, stream, ticks, M, world_t, sender_t, repl_t)
    t_max_ms, pairs_all = reduce_over_ranks(res["t_ms"], res["P"], dev, world_size)
    steps = a.steps
    k_avg_s = res["route_ms"] / res["launches"] / 1e3
    B = algorithmic_bytes(M, res["F"] // steps, res["P"] // steps) + 40 * (res["ops"] // steps)
    update_ms = (res["t_ms"] - res["route_ms"]) / steps
    out = _line(a, world_size, pairs_all / (t_max_ms / 1e3), t_max_ms / steps, "weak",
                f"C4 world-sharded: 8 worlds x 50k peers per GPU ({8 * world_size} worlds in all), 3x3x3 each, "
                "U[-256,256)^3 per world; per tick 5% of peers move N(0,16)^3 (incremental unsub/sub churn), then "
                "one LocalMessage per peer (ExceptSelf)" + ("" if a.scale == 1.0 else f" (scaled {a.scale})"),
                {"messages_per_tick": M * world_size, "peers_per_gpu": M, "subscriptions_per_gpu": int(S0),
                 "churn_ops_per_tick_per_gpu": res["ops"] // steps, "pairs_per_tick": int(pairs_all) // steps,
                 "update_ms_per_tick": round(update_ms, 3), "route_ms_per_tick": round(res["route_ms"] / steps, 3),
                 "incremental_updates": res["incremental"], "rebuild_fallbacks": res["fallbacks"],
                 "parallelism": f"world-sharded x{world_size}", "table_build_s": round(build_s, 3),
                 "generate_s": round(gen_s, 1)},
                {"bound": "hbm", "achieved": B / (t_max_ms / steps / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                 "unit": "GB/s", "frac": B / (t_max_ms / steps / 1e3) / 1e9 / HBM_PEAK_GBS,
                 "traffic": _pmc_tick_traffic("r04_pmc_c4.json", a.scale) if world_size == 1 else None,
                 "kernel": "whole tick (incremental update + route); route launch alone below",
                 "kernel_avg_us": k_avg_s * 1e6, "algorithmic_bytes": B},
                "synthetic (splitmix64, SURVEY.md §8(d) C4 generator)")
    if rank == 0 and world_size == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = _cpu_churn_sample(init, ticks, c4.world, a.cpu_seconds)
    r.close()
    return out


def _cpu_churn_sample(init, ticks, world, seconds):
    """The C restatement on 1 host thread, on ONE world of the GPU's eight (a bounded sample):
    its initial subscriptions (not timed), then whole ticks — that world's churn ops applied one
    by one, then its messages routed — until `seconds` of ticks have run."""
    from oracle import oracle as orc
    w0 = world.min()
    o = orc.COracle(16)
    o.apply_ops(init[init["world"] == w0])
    sel = world == w0
    M = int(sel.sum())
    wz = np.full(M, w0, np.uint32)
    sender = np.flatnonzero(sel).astype(np.uint32)
    repl = np.zeros(M, np.uint8)
    import ctypes
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    offs = np.empty(M + 1, np.uint32)
    cap = 128 * M
    peers = np.empty(cap, np.uint32)
    F = ctypes.c_uint64()
    pairs = n = 0
    t = 0.0
    for ops, pos in ticks:
        mine = np.ascontiguousarray(ops[ops["world"] == w0])
        mpos = np.ascontiguousarray(pos[sel])
        t0 = time.perf_counter()
        o.lib.wqo_apply_ops(o.h, vp(mine), len(mine))
        P = o.lib.wqo_route(o.h, vp(mpos), None, vp(wz), vp(sender), vp(repl), M, vp(offs), vp(peers), cap,
                            ctypes.byref(F))
        t += time.perf_counter() - t0
        pairs += P
        n += 1
        if t >= seconds:
            break
    return {"value": pairs / t, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"C4, world {int(w0)} only (1 of 8 per GPU): {n} whole ticks (churn ops applied in order, "
                      f"then {M} messages routed; {pairs} pairs) in {t:.2f} s by oracle/wq_oracle.c on 1 host thread"}


def run_c5(a, rank, world_size, local_rank, dev):
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Router

    if world_size > 1:
        return _run_c5_sharded(a, rank, world_size, local_rank, dev)
    c5 = synth_ext.config_c5(scale=a.scale)
    t0 = time.perf_counter()
    init = c5.initial_ops()
    init_pos = c5.pos.copy()
    ticks = []
    for _ in range(a.warmup + a.steps):
        ops = c5.step()
        ticks.append((ops, c5.pos.copy()))
    gen_s = time.perf_counter() - t0
    M = c5.n
    stream = torch.cuda.Stream(device=dev)
    r = Router(16, local_rank)
    r.set_stream(stream.cuda_stream)
    t0 = time.perf_counter()
    r.apply_ops(init)
    build_s = time.perf_counter() - t0
    S0 = r.stats()["n_entries"]
    r.set_peer_positions(init_pos)
    r.set_radius(c5.radius)
    world_t = torch.zeros(M, dtype=torch.int32, device=dev)
    sender_t = torch.from_numpy(np.arange(M, dtype=np.int32)).to(dev)
    repl_t = torch.zeros(M, dtype=torch.uint8, device=dev)
    res = _churn_ticks(a, r, dev, stream, ticks, M, world_t, sender_t, repl_t, positions=True)
    steps = a.steps
    k_avg_s = res["route_ms"] / res["launches"] / 1e3
    P, F = res["P"] // steps, res["F"] // steps
    B = algorithmic_bytes(M, F, P) + 40 * (res["ops"] // steps) + 24 * M + 24 * F
    out = _line(a, 1, res["P"] / (res["t_ms"] / 1e3), res["t_ms"] / steps, "strong",
                "C5: 1M entities in U[-1024,1024)^3 moving U[-4,4)^3 per tick, 3x3x3 subscriptions kept current "
                "by incremental churn, one LocalMessage each, exact radius filter r=16 (f64, no FMA) after the "
                "cube broadphase; one GPU" + ("" if a.scale == 1.0 else f" (scaled {a.scale})"),
                {"messages_per_tick": M, "entities": M, "subscriptions": int(S0),
                 "churn_ops_per_tick": res["ops"] // steps, "pairs_per_tick": P, "broadphase_candidates_per_tick": F,
                 "update_ms_per_tick": round((res["t_ms"] - res["route_ms"]) / steps, 3),
                 "route_ms_per_tick": round(res["route_ms"] / steps, 3),
                 "incremental_updates": res["incremental"], "rebuild_fallbacks": res["fallbacks"],
                 "parallelism": "1 GPU", "table_build_s": round(build_s, 3), "generate_s": round(gen_s, 1)},
                {"bound": "hbm", "achieved": B / (res["t_ms"] / steps / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                 "unit": "GB/s", "frac": B / (res["t_ms"] / steps / 1e3) / 1e9 / HBM_PEAK_GBS,
                 "traffic": _pmc_tick_traffic("r04_pmc_c5.json", a.scale),
                 "kernel": "whole tick (incremental update + positions + radius route); route launches alone below",
                 "kernel_avg_us": k_avg_s * 1e6, "algorithmic_bytes": B},
                "synthetic (splitmix64, SURVEY.md §8(d) C5 generator)")
    r.close()
    if not a.no_cpu_baseline:
        tick_ops = [t[0] for t in ticks[:a.warmup + 1]]
        out["cpu_baseline"] = _cpu_c5_measured(init, tick_ops, ticks[a.warmup][1], c5.radius)
        out["cpu_baseline_faithful"] = _cpu_c5_sample(init, tick_ops, ticks[a.warmup][1], c5.radius, a.cpu_seconds)
    return out


def _cpu_c5_measured(init, tick_ops, pos_after, radius):
    """One whole C5 tick MEASURED on 1 host thread by the C restatement in checker mode
    (wqo_set_fast: the same sets, without remove_subscription's O(#cubes) scan of
    area_map.rs:113-116): the tick's churn ops applied in order, then its 1M messages routed with the
    radius filter (wqo_route_radius). The table before the tick is built untimed."""
    import ctypes
    from oracle import oracle as orc
    vp = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    M = len(pos_after)
    o = orc.COracle(16)
    o.set_fast(True)
    o.apply_ops(init)
    for ops in tick_ops[:-1]:
        o.apply_ops(ops)
    ops = np.ascontiguousarray(tick_ops[-1])
    world = np.zeros(M, np.uint32)
    sender = np.arange(M, dtype=np.uint32)
    repl = np.zeros(M, np.uint8)
    offs = np.empty(M + 1, np.uint32)
    pa = np.ascontiguousarray(pos_after)
    t0 = time.perf_counter()
    o.apply_ops(ops)
    t_ops = time.perf_counter() - t0
    t0 = time.perf_counter()
    P = o.lib.wqo_route_radius(o.h, vp(pa), vp(world), vp(sender), vp(repl), M, vp(pa), M, float(radius),
                               vp(offs), None, 0, None)
    t_route = time.perf_counter() - t0
    o.close()
    return {"value": P / (t_ops + t_route), "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"one whole C5 tick measured: {len(ops)} churn ops applied in {t_ops:.2f} s and {M} messages "
                      f"routed with the radius filter in {t_route:.2f} s ({P} pairs), oracle/wq_oracle.c in checker "
                      f"mode (the reference's sets without its O(#cubes) unsubscribe scan; see "
                      f"cpu_baseline_faithful for that scan) on 1 host thread"}


def _cpu_c5_sample(init, tick_ops, pos_after, radius, seconds):
    """C5 on 1 host thread by the C restatement, one whole tick estimated from two timed parts:
      route  the tick's 1M messages with the radius filter (wqo_route_radius), on a table brought
             to the tick's state in checker mode (wqo_set_fast; the route itself is the same code);
      churn  a strided sample of the tick's ops applied to a FAITHFUL table (the reference's
             O(#cubes) scan per unsubscribe, area_map.rs:113-116), scaled to all of the tick's ops.
    value = pairs of the tick / (t_route + n_ops * t_per_op). The tables are built untimed."""
    import ctypes
    from oracle import oracle as orc
    vp = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    M = len(pos_after)
    fast = orc.COracle(16)
    fast.set_fast(True)
    fast.apply_ops(init)
    for ops in tick_ops:  # the table as the first timed tick sees it
        fast.apply_ops(ops)
    world = np.zeros(M, np.uint32)
    sender = np.arange(M, dtype=np.uint32)
    repl = np.zeros(M, np.uint8)
    offs = np.empty(M + 1, np.uint32)
    t0 = time.perf_counter()
    P = fast.lib.wqo_route_radius(fast.h, vp(np.ascontiguousarray(pos_after)), vp(world), vp(sender), vp(repl), M,
                                  vp(np.ascontiguousarray(pos_after)), M, float(radius), vp(offs), None, 0, None)
    t_route = time.perf_counter() - t0
    fast.close()
    faith = orc.COracle(16)
    faith.apply_ops(init)
    n_ops = len(ops)
    stride = max(1, n_ops // 4096)
    sample = np.ascontiguousarray(ops[::stride])
    done, t_ops = 0, 0.0
    while done < len(sample) and t_ops < seconds / 2:
        chunk = sample[done:done + 64]
        t0 = time.perf_counter()
        faith.apply_ops(chunk)
        t_ops += time.perf_counter() - t0
        done += len(chunk)
    faith.close()
    t_tick = t_route + n_ops * (t_ops / done)
    # an estimate, not a measured tick: the churn part is a sample scaled to the whole tick
    return {"value": P / t_tick, "unit": "pairs/s", "cores": 1, "kind": "estimate",
            "sample": f"C5 tick estimate: {M} messages routed with the radius filter in {t_route:.2f} s "
                      f"({P} pairs) + {done} of the tick's {n_ops} churn ops (every {stride}th) applied with the "
                      f"reference's O(#cubes) unsubscribe scan in {t_ops:.2f} s, scaled to all {n_ops} ops: "
                      f"{t_tick:.1f} s per tick, oracle/wq_oracle.c on 1 host thread"}


def _run_c5_sharded(a, rank, world_size, local_rank, dev):
    """C5 over G GPUs by cube hash (strong scaling) through the C ABI's sharded tick: every rank
    applies the churn ops of the cubes it owns (wq_apply_ops_device on its slice of the op stream)
    and holds every entity's position; it ingests 1/G of the messages: 20-byte slots to the owners
    (RCCL), row references + cube-list pools back, filtered by radius on the ingesting GPU."""
    import torch
    from worldql_server_amd import synth_ext
    from worldql_server_amd.router import Router

    c5 = synth_ext.config_c5(scale=a.scale)
    t0 = time.perf_counter()
    init = c5.initial_ops()
    init_pos = c5.pos.copy()
    ticks = []
    for _ in range(a.warmup + a.steps):
        ops = c5.step()
        ticks.append((ops, c5.pos.copy()))
    gen_s = time.perf_counter() - t0
    N = c5.n
    lo, hi = rank * N // world_size, (rank + 1) * N // world_size
    M = hi - lo
    stream = torch.cuda.Stream(device=dev)
    r = Router(16, local_rank)
    r.set_stream(stream.cuda_stream)
    attach_rccl(r, rank, world_size)
    r.sharded_apply_ops(init)
    r.set_peer_positions(init_pos)
    r.set_radius(c5.radius)
    own_ops = []
    for ops, _ in ticks:  # the churn of the cubes this rank owns (host-partitioned on ingest)
        owner = r.shard_ops(ops, world_size)
        own_ops.append(_ops_tensor(ops[owner == rank], dev))
    pos_d = [torch.from_numpy(p_).to(dev) for _, p_ in ticks]
    world = torch.zeros(M, dtype=torch.int32, device=dev)
    sender = torch.arange(lo, hi, dtype=torch.int32, device=dev)
    repl = torch.zeros(M, dtype=torch.uint8, device=dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = 16 * M + 1024
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    state = {"i": 0}
    cnt = torch.zeros((a.warmup + a.steps, 24), dtype=torch.uint8, device=dev)

    def one():
        i = state["i"]
        r.apply_ops_device(own_ops[i].data_ptr(), int(own_ops[i].shape[0]) // 40)
        r.set_peer_positions_device(pos_d[i].data_ptr(), N)
        p = pos_d[i][lo:hi]
        # asynchronous sharded tick: P and the status bits of tick i land in cnt[i]
        r.sharded_route_async(p.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M,
                              offs.data_ptr(), peers.data_ptr(), msgs.data_ptr(), cap, cnt[i].data_ptr())
        state["i"] = i + 1

    for _ in range(a.warmup):
        one()
    t_ms = timed_ticks(one, a.steps, stream, dev, world_size, [r])
    c = _counters(cnt)[a.warmup:]
    assert (c["error"] == 0).all() and (c["overflow"] == 0).all(), c
    t_max_ms, pairs_all = reduce_over_ranks(t_ms, int(c["n_pairs"].sum()), dev, world_size)
    out = _line(a, world_size, pairs_all / (t_max_ms / 1e3), t_max_ms / a.steps, "strong",
                f"C5 over {world_size} GPUs by cube hash: 1M entities, incremental churn on the owners, "
                "slots to the owners and cube-list pools back by RCCL (wq_sharded_route_tick_device), exact radius "
                "filter r=16 on the ingesting GPU"
                + ("" if a.scale == 1.0 else f" (scaled {a.scale})"),
                {"messages_per_tick": N, "messages_per_gpu": M, "entities": N,
                 "pairs_per_tick": int(pairs_all) // a.steps,
                 "parallelism": f"cube-hash x{world_size} (RCCL all-to-all)", "generate_s": round(gen_s, 1)},
                {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                 "traffic": None, "kernel": "whole sharded tick (update + exchange + radius route)"},
                "synthetic (splitmix64, SURVEY.md §8(d) C5 generator)")
    r.close()
    return out
