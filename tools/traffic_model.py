"""Calibrated HBM bytes of a tick from rocprofv3 FETCH_SIZE / WRITE_SIZE (round-4 calibration,
tools/fetchcal.hip -> profiles/r04_fetch_calibration.json).

What the calibration showed on gfx950 (4 GiB buffer, byte counts known by construction):
  * FETCH_SIZE = 64 B x TCC_EA0_RDREQ, whatever the access;
  * a wide coalesced streaming read (4 or 16 B per lane) issues one request per 128-B line and is
    tallied at half (fetch / requested = 0.500 for stream4_rd and stream16_rd);
  * a random access to a part of a line is ONE request (rdreq / access = 1.0 for 32, 64 and 128 B
    of a line) tallied at 64 B; for a whole-line read that is half the line, for a 32- or 64-B read
    it is the 64-B sector the access lies in;
  * WRITE_SIZE reads the bytes exactly for 4- and 16-B-per-lane streaming stores (1.000).
So a kernel's read traffic is FETCH x 2 when its requests are whole lines (streaming reads, whole
record lines, list runs) and FETCH + (its streaming read bytes) / 2 when its random requests are
partial-line (<= 64 B) reads: the count pass (32 B of each record line) and the churn events pass
(12 B of each record line). The streaming bytes of those two are known from the workload sizes.
This replaces the blanket FETCH x 2 of rounds 1-3, which double-counted the partial-line reads.

    python tools/traffic_model.py            # re-derives the committed PMC summaries, prints them
"""
from __future__ import annotations

import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# kernel-name substring -> streaming read bytes per dispatch, for the kernels whose random reads are
# partial-line requests; every other kernel reads whole lines (or streams): FETCH x 2
PARTIAL = {
    "count_kernel": lambda z: 33 * z["M"],       # pos 24 + world 4 + sender 4 + repl 1 per message
    "k_delta_events": lambda z: 40 * z["ops"],   # the 40-byte ops
}


def kernel_read_bytes(kernel: str, fetch_bytes_raw: float, sizes: dict) -> float:
    """Calibrated read bytes of one dispatch (or per-tick sum) of `kernel` from its raw FETCH bytes
    (FETCH_SIZE KB x 1024, not doubled)."""
    for key, stream in PARTIAL.items():
        if key in kernel and "radius" not in kernel:
            return fetch_bytes_raw + stream(sizes) / 2
    return 2 * fetch_bytes_raw


def route_tick_traffic(pmc: dict, exclude: str = "") -> dict:
    """A route PMC summary (tools/pmc_summary.py: per-kernel means of FETCH_SIZE / WRITE_SIZE in KB
    per dispatch, one dispatch of each kernel per tick) -> calibrated bytes per tick."""
    sizes = {"M": pmc["messages_per_tick"], "P": pmc["pairs_per_tick"]}
    rd = wr = 0.0
    per = {}
    for k, c in pmc["kernels"].items():
        if exclude and exclude in k:
            continue
        r = kernel_read_bytes(k, c.get("FETCH_SIZE", 0.0) * 1024, sizes)
        w = c.get("WRITE_SIZE", 0.0) * 1024
        per[k] = {"read": r, "write": w}
        rd += r
        wr += w
    return {"read": rd, "write": wr, "total": rd + wr, "kernels": per}


def churn_tick_traffic(pmc: dict, ops_per_tick: int, M: int) -> dict:
    """A churn PMC summary (tools/pmc_churn_summary.py: per tick, FETCH already x 2 x 1024 in bytes,
    WRITE x 1024) -> calibrated bytes per tick."""
    sizes = {"M": M, "ops": ops_per_tick}
    rd = wr = 0.0
    per = {}
    for k, c in pmc["kernels"].items():
        r = kernel_read_bytes(k, c.get("FETCH_SIZE", 0.0) / 2, sizes)
        w = c.get("WRITE_SIZE", 0.0)
        per[k] = {"read": r, "write": w}
        rd += r
        wr += w
    return {"read": rd, "write": wr, "total": rd + wr, "kernels": per}


def load(name: str):
    p = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def main():
    out = {}
    for name, ex in (("r02_pmc_route.json", ""), ("r03_pmc_route_c3.json", "tick_kernel")):
        d = load(name)
        if d:
            t = route_tick_traffic(d, ex)
            out[name] = {"M": d["messages_per_tick"], "P": d["pairs_per_tick"], "blanket_x2": d["hbm_bytes_per_launch"],
                         "calibrated": t["total"], "read": t["read"], "write": t["write"]}
    for name, ops, M in (("r03_pmc_c5.json", 6420000, 1000000), ("r02_pmc_c4.json", 632000, 400000)):
        d = load(name)
        if d:
            t = churn_tick_traffic(d, ops, M)
            out[name] = {"blanket_x2": d["hbm_bytes_per_tick"], "calibrated": t["total"], "read": t["read"],
                         "write": t["write"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
