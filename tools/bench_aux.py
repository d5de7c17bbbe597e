#!/usr/bin/env python3
"""Timings of the paths next to the tick on one MI355X:
  F2  per-peer send lists of a C2 tick (10M pairs, 70% of peers connected)
  F3  REMOVE_PEER of 1% / 10% of the peers on a C4 GPU's table (8 worlds x 50k peers, 10.8M entries)
  F1  1,000 GlobalMessages to C4 worlds (each reaching a whole world's 50k peers)
  and the C2 tick through the host-array entry point (PCIe-inclusive)
Device time with HIP events on the router's stream; one JSON line per measurement."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from worldql_server_amd import abi, synth, synth_ext
    from worldql_server_amd.router import Router
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)

    def timed(fn, reps=5):
        fn()
        s.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(reps):
            e0.record(s)
            fn()
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    # F2 on C2
    w = synth.config_c2()
    r = Router(16, 0)
    r.set_stream(s.cuda_stream)
    r.apply_ops(w.ops)
    with torch.cuda.stream(s):
        pos = torch.from_numpy(w.pos).to(dev)
        wo = torch.from_numpy(w.world.view(np.int32)).to(dev)
        se = torch.from_numpy(w.sender.view(np.int32)).to(dev)
        rp = torch.from_numpy(w.repl).to(dev)
        M = len(w.world)
        offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
        peers = torch.empty(12 * M, dtype=torch.int32, device=dev)
        cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
        r.route_device(pos.data_ptr(), wo.data_ptr(), se.data_ptr(), rp.data_ptr(), M, offs.data_ptr(),
                       peers.data_ptr(), None, 12 * M, cnt.data_ptr())
        s.synchronize()
        P = int(cnt.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]["n_pairs"])
        N = w.n_peers
        bits = np.random.default_rng(1).random(((N + 31) // 32) * 32) < 0.7
        conn = torch.from_numpy(np.packbits(bits, bitorder="little").view(np.int32)).to(dev)
        po = torch.empty(N + 1, dtype=torch.int32, device=dev)
        mo = torch.empty(P, dtype=torch.int32, device=dev)
        ms = timed(lambda: r.peer_major_device(offs.data_ptr(), peers.data_ptr(), M, P, conn.data_ptr(), N,
                                               po.data_ptr(), mo.data_ptr()))
    print(json.dumps({"path": "F2 per-peer send lists", "workload": "C2 tick", "pairs": P, "peers": N,
                      "connected": 0.7, "ms": round(ms, 3), "pairs_per_s": P / ms * 1e3}), flush=True)
    # the host-array boundary: wq_route_tick copies the inputs in and the CSR out over PCIe
    r.set_stream(None)
    out = r.route(w.pos, w.world, w.sender, w.repl, with_msgs=True)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        out = r.route(w.pos, w.world, w.sender, w.repl, with_msgs=True)
        ts.append((time.perf_counter() - t0) * 1e3)
    ms = float(np.median(ts))
    print(json.dumps({"path": "C2 tick through the host-array ABI (wq_route_tick: H2D inputs, D2H offsets, peers, msgs), pageable numpy arrays",
                      "pairs": len(out[1]), "ms_wall": round(ms, 3), "pairs_per_s": len(out[1]) / ms * 1e3,
                      "bytes_moved": int(M * 33 + (M + 1) * 4 + 8 * len(out[1]))}), flush=True)
    import ctypes
    from worldql_server_amd.router import PinnedArray
    Pn = len(out[1])
    pin = {k: PinnedArray(v.shape, v.dtype) for k, v in
           (("pos", w.pos), ("world", w.world), ("sender", w.sender), ("repl", w.repl))}
    for k, v in (("pos", w.pos), ("world", w.world), ("sender", w.sender), ("repl", w.repl)):
        pin[k].array[...] = v
    o_off, o_peers, o_msgs = PinnedArray((M + 1,), np.uint32), PinnedArray((Pn,), np.uint32), PinnedArray((Pn,), np.uint32)
    n = ctypes.c_size_t()
    vp = lambda a: ctypes.c_void_p(a.ptr.value)
    ts = []
    for _ in range(6):
        t0 = time.perf_counter()
        rc = r.lib.wq_route_tick(r.h, vp(pin["pos"]), None, vp(pin["world"]), vp(pin["sender"]), vp(pin["repl"]), M,
                                 vp(o_off), vp(o_peers), vp(o_msgs), Pn, ctypes.byref(n))
        ts.append((time.perf_counter() - t0) * 1e3)
        assert rc == 0 and n.value == Pn
    assert (o_peers.array == out[1]).all()
    ms = float(np.median(ts[1:]))
    print(json.dumps({"path": "C2 tick through the host-array ABI, pinned buffers (wq_host_alloc)", "pairs": Pn,
                      "ms_wall": round(ms, 3), "pairs_per_s": Pn / ms * 1e3,
                      "GB_per_s_pcie": (M * 33 + (M + 1) * 4 + 8 * Pn) / ms / 1e6}), flush=True)
    for a in list(pin.values()) + [o_off, o_peers, o_msgs]:
        a.close()
    r.close()

    # F3 and F1 on a C4 GPU's table
    c4 = synth_ext.config_c4(1.0, worlds=range(8))
    init = c4.initial_ops()
    warm = Router(16, 0)  # first use of the REMOVE_PEER kernels loads their code object: not timed
    warm.apply_ops(init[:27])
    warm.remove_peers(np.array([0], np.uint32))
    warm.close()
    for frac in (0.01, 0.10):
        r = Router(16, 0)
        r.set_stream(s.cuda_stream)
        r.apply_ops(init)
        S = r.stats()["n_entries"]
        gone = np.random.default_rng(2).choice(c4.n_peers, int(frac * c4.n_peers), replace=False).astype(np.uint32)
        s.synchronize()
        t0 = time.perf_counter()
        r.remove_peers(gone)
        s.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        S1 = r.stats()["n_entries"]
        print(json.dumps({"path": "F3 REMOVE_PEER in place", "workload": "C4 GPU table (8 worlds x 50k peers)",
                          "entries": int(S), "peers_removed": len(gone), "entries_removed": int(S - S1),
                          "ms_wall": round(ms, 3)}), flush=True)
        if frac == 0.01:
            Mg = 1000
            g = np.random.default_rng(3)
            gw = torch.from_numpy(g.integers(0, 8, Mg).astype(np.int32)).to(dev)
            gs = torch.from_numpy(g.integers(0, c4.n_peers, Mg).astype(np.int32)).to(dev)
            gr = torch.zeros(Mg, dtype=torch.uint8, device=dev)
            goffs = torch.empty(Mg + 1, dtype=torch.int32, device=dev)
            gcap = Mg * 50_000
            gpeers = torch.empty(gcap, dtype=torch.int32, device=dev)
            gcnt = torch.zeros(24, dtype=torch.uint8, device=dev)
            r.stats()  # any-keys regenerated outside the timing
            with torch.cuda.stream(s):
                ms = timed(lambda: r.route_global_device(gw.data_ptr(), gs.data_ptr(), gr.data_ptr(), Mg,
                                                         goffs.data_ptr(), gpeers.data_ptr(), None, gcap,
                                                         gcnt.data_ptr()))
            Pg = int(gcnt.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]["n_pairs"])
            print(json.dumps({"path": "F1 GlobalMessage", "workload": "1000 messages to C4 worlds", "pairs": Pg,
                              "ms": round(ms, 3), "pairs_per_s": Pg / ms * 1e3,
                              "GB_per_s_written": Pg * 4 / ms / 1e6}), flush=True)
        r.close()


if __name__ == "__main__":
    main()
