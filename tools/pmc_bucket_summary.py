"""Per-kernel SQ counters of the churn kernels from tools/pmc_bucket.sh (one rocprofv3 --pmc pass per
counter group), averaged per dispatch, with the dispatch's resources and per-wave instruction counts.
    python tools/pmc_bucket_summary.py gpurun_out/pmcb_c5 [--json profiles/r06_pmc_c5_bucket_sq.json]"""
import argparse
import collections
import csv
import glob
import json
import os

KERNELS = ("k_delta_bucket", "k_delta_events", "k_sort_scatter", "k_sort_hist")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(a.root, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            for k in KERNELS:
                if k in r["Kernel_Name"]:
                    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    meta[k] = {"grid": int(r["Grid_Size"]), "workgroup": int(r["Workgroup_Size"]),
                               "lds_bytes": int(r["LDS_Block_Size"]), "vgpr": int(r["VGPR_Count"]),
                               "sgpr": int(r["SGPR_Count"]), "kernel": r["Kernel_Name"][:80]}
    out = {}
    for k, d in acc.items():
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        row = dict(meta[k])
        row["per_dispatch"] = {c: round(v) for c, v in avg.items()}
        waves = avg.get("SQ_WAVES")
        if waves:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                if c in avg:
                    row.setdefault("per_wave", {})[c] = round(avg[c] / waves, 1)
        if avg.get("SQ_WAVE_CYCLES"):
            wc = avg["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
                if c in avg:
                    row.setdefault("frac_of_wave_cycles", {})[c] = round(avg[c] / wc, 3)
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_bank_conflict_frac"] = round(avg.get("SQ_LDS_BANK_CONFLICT", 0) / avg["SQ_LDS_IDX_ACTIVE"], 3)
        out[k] = row
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.json:
        with open(a.json, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
