#!/usr/bin/env python3
"""Summarise a rocprofv3 run directory (profiles/run_prof.sh) into <out>.json + <out>.md:
per-kernel average duration (kernel trace stats) and per-launch PMC values of the report
kernel.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB;
FETCH_SIZE under-reads wide coalesced streams by 2x on gfx950 (applied as an upper bound;
narrow accesses are uncalibrated), WRITE_SIZE is taken as is."""
import csv
import collections
import json
import sys


def main(src, out, alg_bytes=None):
    stats = list(csv.DictReader(open(f"{src}/trace/run_kernel_stats.csv")))
    pmc = collections.defaultdict(list)
    import glob
    import os
    for part in sorted(os.path.basename(p) for p in glob.glob(f"{src}/pmc_*") if os.path.isdir(p)):
        try:
            for r in csv.DictReader(open(f"{src}/{part}/run_counter_collection.csv")):
                if "report_kernel" in r["Kernel_Name"]:
                    pmc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        except FileNotFoundError:
            pass
    per = {k: sum(v) / len(v) for k, v in pmc.items()}
    fetch = per.get("FETCH_SIZE", 0) * 1024
    write = per.get("WRITE_SIZE", 0) * 1024
    res = {
        "kernels": [{"name": s["Name"], "calls": int(s["Calls"]), "avg_ns": float(s["AverageNs"]),
                     "pct": float(s["Percentage"])} for s in stats],
        "report_kernel_pmc_per_launch": per,
        "hbm_fetch_bytes_raw": fetch, "hbm_write_bytes": write,
        "hbm_bytes_per_launch": 2 * fetch + write,
        "hbm_bytes_note": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving applied; narrow loads uncalibrated)",
    }
    if "SQ_LDS_BANK_CONFLICT" in per and per.get("SQ_LDS_IDX_ACTIVE"):
        res["lds_bank_conflict_frac"] = per["SQ_LDS_BANK_CONFLICT"] / per["SQ_LDS_IDX_ACTIVE"]
    if alg_bytes:
        res["alg_bytes_per_launch"] = alg_bytes
    json.dump(res, open(out + ".json", "w"), indent=1)
    with open(out + ".md", "w") as f:
        f.write(f"# rocprofv3 summary: {src}\n\n| kernel | calls | avg us | % |\n|---|---|---|---|\n")
        for k in res["kernels"]:
            f.write(f"| {k['name'][:70]} | {k['calls']} | {k['avg_ns'] / 1000:.1f} | {k['pct']:.2f} |\n")
        f.write("\nreport_kernel PMC per launch:\n\n")
        for k, v in sorted(per.items()):
            f.write(f"- {k}: {v:,.1f}\n")
        f.write(f"\nHBM bytes per launch (2*FETCH + WRITE): {res['hbm_bytes_per_launch'] / 1e6:.1f} MB\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None)
