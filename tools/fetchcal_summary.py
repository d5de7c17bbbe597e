"""Summarise tools/fetchcal.sh: per access shape, what the counters report against the bytes the
shape requests by construction (tools/fetchcal.hip), -> profiles/r04_fetch_calibration.json.

    python tools/fetchcal_summary.py gpurun_out/fetchcal profiles/r04_fetch_calibration.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main():
    root, out = sys.argv[1], sys.argv[2]
    plain = json.load(open(os.path.join(root, "plain.json")))
    per = load(root)  # kernel short name -> counter -> values (one per dispatch)
    rows = {}
    for s in plain["shapes"]:
        rows[s["shape"]] = dict(s)
    # line_rd<2>, <4>, <8> share a base name: match by template argument
    for k, cs in per.items():
        base = k.split("(")[0]
        shape = {"line_rd<2>": "line32_rd", "line_rd<4>": "line64_rd", "line_rd<8>": "line128_rd"}.get(base, base)
        if shape not in rows:
            continue
        r = rows[shape]
        for c, v in cs.items():
            r[c] = min(v)  # one dispatch per pass (fetchcal 1)
        req = r["requested_bytes"]
        lines = r["lines_distinct"]
        if "FETCH_SIZE" in r:
            fb = r["FETCH_SIZE"] * 1024
            r["fetch_bytes"] = fb
            r["fetch_over_requested"] = fb / req
            r["fetch_per_distinct_line"] = fb / lines
        if "WRITE_SIZE" in r:
            r["write_over_requested"] = r["WRITE_SIZE"] * 1024 / req
        if "TCC_EA0_RDREQ_sum" in r:
            r["rdreq_per_distinct_line"] = r["TCC_EA0_RDREQ_sum"] / lines
            r["rdreq_per_unit"] = r["TCC_EA0_RDREQ_sum"] / r["units"]  # per lane access / per run
            r["rdreq_32B_share"] = r.get("TCC_EA0_RDREQ_32B_sum", 0.0) / max(r["TCC_EA0_RDREQ_sum"], 1.0)
        if "FETCH_SIZE" in r:
            r["fetch_per_unit"] = r["FETCH_SIZE"] * 1024 / r["units"]
        if "TCC_HIT_sum" in r:
            r["tcc_hit_per_unit"] = r["TCC_HIT_sum"] / r["units"]
    doc = {"source": "tools/fetchcal.hip + tools/fetchcal.sh (rocprofv3 --pmc, one group per pass), buffer "
                     f"{plain['buffer_bytes']} B", "shapes": list(rows.values())}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for r in rows.values():
        print(f"{r['shape']:12s} req {r['requested_bytes']:.3g} B  fetch/req {r.get('fetch_over_requested', float('nan')):.3f}"
              f"  fetch/unit {r.get('fetch_per_unit', float('nan')):.1f}  rdreq/unit "
              f"{r.get('rdreq_per_unit', float('nan')):.2f}  hit/unit {r.get('tcc_hit_per_unit', float('nan')):.2f}"
              f"  write/req {r.get('write_over_requested', float('nan')):.3f}  {r['requested_GBps']:.0f} GB/s req")


if __name__ == "__main__":
    main()
