"""Times every compiled route-kernel shape on the C2 tick (kernel-only HIP events) and checks
that all shapes produce identical outputs. Usage: python tools/tune_route.py [--scale S] [--workload c2|c3]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--cfgs", default="0,1,2,3,4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-check", action="store_true", help="timing-only configs (wrong outputs)")
    ap.add_argument("--raw-keys", action="store_true", help="route pre-quantised keys (skips kernel 1)")
    ap.add_argument("--slack", type=int, default=8, help="record slots per cube (wq_debug_set_record_slack)")
    ap.add_argument("--workload", choices=["c2", "c3"], default="c2")
    a = ap.parse_args()
    import torch
    from worldql_server_amd import abi, synth
    from worldql_server_amd.router import Router
    dev = torch.device("cuda:0")
    if a.workload == "c3":
        from worldql_server_amd import synth_ext
        w = synth_ext.config_c3(scale=a.scale)
    else:
        w = synth.config_c2(scale=a.scale)
    M = len(w.world)
    r = Router(16, 0)
    s = torch.cuda.Stream(device=dev)
    r.set_stream(s.cuda_stream)
    r.set_record_slack(a.slack)
    r.apply_ops(w.ops)
    pos = torch.from_numpy(w.pos).to(dev)
    world = torch.from_numpy(w.world.view(np.int32)).to(dev)
    sender = torch.from_numpy(w.sender.view(np.int32)).to(dev)
    repl = torch.from_numpy(w.repl).to(dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = 12 * M
    if a.workload == "c3":  # heavy fan-out: size the outputs with a counts-only call
        cnt0 = torch.zeros(24, dtype=torch.uint8, device=dev)
        r.route_device(pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
                       0, 0, 0, cnt0.data_ptr())
        torch.cuda.synchronize()
        cap = int(cnt0.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]["n_pairs"]) + 1024
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = torch.zeros(24, dtype=torch.uint8, device=dev)
    keys = None
    if a.raw_keys:
        keys = torch.empty((M, 3), dtype=torch.int64, device=dev)
        r.lib.wq_quantize_device(r.h, pos.data_ptr(), 3 * M, keys.data_ptr())
    torch.cuda.synchronize()
    ref = None
    res, phases = {}, {}
    cfgs = [int(c) for c in a.cfgs.split(",")]
    for rnd in range(a.rounds):
        for cfg in cfgs:
            r.set_route_config(cfg)
            args = (0 if a.raw_keys else pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M,
                    offs.data_ptr(), peers.data_ptr(), msgs.data_ptr(), cap)
            kw = {"keys_ptr": keys.data_ptr()} if a.raw_keys else {}
            for _ in range(3):
                r.route_device(*args, cnt.data_ptr(), **kw)
            torch.cuda.synchronize()
            c = cnt.cpu().numpy().view(abi.COUNTERS_DTYPE)[0]
            P = int(c["n_pairs"])
            h = (offs.clone(), peers[:P].clone(), msgs[:P].clone())  # compared on the device
            if ref is None:
                ref = h
            assert a.no_check or all(torch.equal(x, y) for x, y in zip(h, ref)), f"cfg {cfg} differs"
            del h
            r.profile_enable(True)
            for _ in range(a.steps):
                r.route_device(*args, **kw)
            ms, n, ph, nph = r.profile_read_phases()
            r.profile_enable(False)
            res.setdefault(cfg, []).append(ms / n * 1e3)
            if nph:
                phases.setdefault(cfg, []).append([round(x / nph * 1e3, 1) for x in ph])
    print(json.dumps({"M": M, "P": P, "us_per_launch": {k: [round(x, 2) for x in v] for k, v in res.items()},
                      "count_scan_emit_us": phases, "sclk_mhz": round(r.probe_sclk(), 1)}))


if __name__ == "__main__":
    main()
