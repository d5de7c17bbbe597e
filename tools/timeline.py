"""Per-block phase timeline of the single-launch tick on the C2 (or C3) workload (s_memrealtime, 100 MHz).
Prints percentiles over blocks of: start offset, count phase, prefix wait, emit phase, end offset.
Usage: python tools/timeline.py [--cfg N] [--scale S] [--workload c2|c3]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=0)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--dump", default="")
    ap.add_argument("--workload", choices=["c2", "c3"], default="c2")
    a = ap.parse_args()
    import torch
    from worldql_server_amd import synth
    from worldql_server_amd.router import Router
    dev = torch.device("cuda:0")
    if a.workload == "c3":
        from worldql_server_amd import synth_ext
        w = synth_ext.config_c3(scale=a.scale)
    else:
        w = synth.config_c2(scale=a.scale)
    M = len(w.world)
    r = Router(16, 0)
    r.set_stream(torch.cuda.current_stream(dev).cuda_stream)  # stamps are zeroed on this stream
    r.set_route_config(a.cfg)
    r.apply_ops(w.ops)
    pos = torch.from_numpy(w.pos).to(dev)
    world = torch.from_numpy(w.world.view(np.int32)).to(dev)
    sender = torch.from_numpy(w.sender.view(np.int32)).to(dev)
    repl = torch.from_numpy(w.repl).to(dev)
    offs = torch.empty(M + 1, dtype=torch.int32, device=dev)
    cap = (50 if a.workload == "c3" else 12) * M
    peers = torch.empty(cap, dtype=torch.int32, device=dev)
    msgs = torch.empty(cap, dtype=torch.int32, device=dev)
    stamps = torch.zeros(4 * 65536, dtype=torch.int64, device=dev)
    args = (pos.data_ptr(), world.data_ptr(), sender.data_ptr(), repl.data_ptr(), M, offs.data_ptr(),
            peers.data_ptr(), msgs.data_ptr(), cap)
    for _ in range(5):
        r.route_device(*args)
    r.lib.wq_debug_set_timeline(r.h, stamps.data_ptr())
    rows, raw = [], []
    for _ in range(5):
        stamps.zero_()
        r.route_device(*args)
        torch.cuda.synchronize()
        s = stamps.cpu().numpy().reshape(-1, 4)
        s = s[s[:, 0] > 0].astype(np.float64)
        raw.append(s)
        t0 = s[:, 0].min()
        rows.append(np.stack([s[:, 0] - t0, s[:, 1] - s[:, 0], s[:, 2] - s[:, 1], s[:, 3] - s[:, 2], s[:, 3] - t0], 1))
    r.lib.wq_debug_set_timeline(r.h, None)
    x = np.concatenate(rows) / 100.0  # 100 MHz ticks -> us
    print(f"blocks {len(x) // 5}; microseconds, percentiles over blocks and 5 ticks")
    for i, nm in enumerate(["start", "count", "wait", "emit", "end"]):
        q = np.percentile(x[:, i], [0, 10, 50, 90, 100])
        print(f"  {nm:6s} " + "  ".join(f"{v:7.1f}" for v in q))
    s = raw[-1]
    nb = len(s)
    cnt = (s[:, 1] - s[:, 0]) / 100.0
    st = (s[:, 0] - s[:, 0].min()) / 100.0
    b = np.arange(nb)
    print("count phase by b % 8:", " ".join(f"{cnt[b % 8 == k].mean():5.1f}" for k in range(8)))
    q = np.array_split(np.arange(nb), 8)
    print("count phase by block octile:", " ".join(f"{cnt[i].mean():5.1f}" for i in q))
    print("start by block octile:", " ".join(f"{st[i].mean():5.1f}" for i in q))
    if a.dump:
        np.save(a.dump, raw[-1])


if __name__ == "__main__":
    main()
