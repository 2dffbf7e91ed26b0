#!/usr/bin/env python3
"""Summarise a profiles/run_prof.sh directory into <out>.json + <out>.md: per-kernel average
duration (rocprofv3 kernel-trace stats), per-launch PMC values of every pw:: kernel, and the
HBM traffic of one pass of the hot path (all kernels of pw_report_events + pw_stop_table_build,
or of the GapAssem calls).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so traffic is taken as
2*FETCH + WRITE.  Round 6 calibrated the factor on the patterns these kernels use
(profiles/calib/fetch_calib.hip, profiles/r6_calib/calibration.md: 2 GiB buffers, known bytes):
FETCH_SIZE is exactly 1/2 of the 128-B line fills for coalesced 16 B/lane streams, 4 B and 16 B
per-lane gathers (one lane per line) and 48-byte per-lane windows alike — every L2 miss fetches a
whole 128-B line and is tallied at 64 B — so 2*FETCH is the memory-side read traffic of every
read pattern here (L2 misses: Infinity-Cache hits included).  WRITE_SIZE is exact for streaming
stores and counts a 32-B sector for each partial-line store.

Occupancy (achieved waves per SIMD, per kernel) = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8) /
(4 * CUs): SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md, SQ PMC units) summed over every
wave, GRBM_GUI_ACTIVE counts busy cycles summed over the 8 XCDs."""
import collections
import csv
import glob
import json
import os
import sys


N_CU = 256


def kname(n):
    """pw::render_kernel from "void pw::render_kernel<true>(pw_report_args, pw::Work)" (templates)."""
    n = n.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n.split("<")[0]


def main(src, out, bench_args=""):
    stats = list(csv.DictReader(open(f"{src}/trace/run_kernel_stats.csv")))
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{src}/pmc_*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            pmc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    per = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in pmc.items()}
    kern = [{"name": kname(s["Name"]), "calls": int(s["Calls"]), "avg_us": float(s["AverageNs"]) / 1000,
             "pct": float(s["Percentage"])} for s in stats]
    pw = [k for k in kern if k["name"].startswith("pw::")]
    fetch = sum(per[k].get("FETCH_SIZE", 0) for k in per) * 1024
    write = sum(per[k].get("WRITE_SIZE", 0) for k in per) * 1024
    a = bench_args.split()
    res = {
        "bench_args": bench_args,
        "config": int(a[a.index("--config") + 1]) if "--config" in a else 2,
        "kernels": kern,
        "pass_us": sum(k["avg_us"] for k in pw),
        "pmc_per_launch": per,
        "hbm_fetch_bytes_raw": fetch,
        "per_kernel_bytes": {k: {"read": 2 * c.get("FETCH_SIZE", 0) * 1024, "write": c.get("WRITE_SIZE", 0) * 1024}
                             for k, c in per.items() if "FETCH_SIZE" in c or "WRITE_SIZE" in c},
        "hbm_write_bytes": write,
        "hbm_bytes_per_launch": 2 * fetch + write,
        "hbm_bytes_note": "one pass = one launch of every pw:: kernel; 2*FETCH_SIZE + WRITE_SIZE (KiB -> bytes; "
                          "the factor 2 calibrated for every read pattern here: profiles/r6_calib/calibration.md)",
    }
    for k, c in per.items():
        if c.get("SQ_LDS_IDX_ACTIVE"):
            c["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
        if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_WAVE_CYCLES"):
            c["occupancy_waves_per_simd"] = 4 * c["SQ_WAVE_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8) / (4 * N_CU)
    res["occupancy_waves_per_simd"] = {k: round(c["occupancy_waves_per_simd"], 2) for k, c in per.items()
                                       if "occupancy_waves_per_simd" in c}
    # the bench's HIP-event bracket covers pw_report_events only (the stop table is built before it)
    rep = [k for k in per if not k.startswith("pw::stop_table")]
    res["hbm_bytes_per_report_pass"] = sum(2 * per[k].get("FETCH_SIZE", 0) + per[k].get("WRITE_SIZE", 0) for k in rep) * 1024
    res["report_pass_us"] = sum(k["avg_us"] for k in pw if not k["name"].startswith("pw::stop_table"))
    json.dump(res, open(out + ".json", "w"), indent=1)
    with open(out + ".md", "w") as f:
        f.write(f"# rocprofv3 summary: {os.path.basename(src)}\n\n| kernel | calls | avg us | % |\n|---|---|---|---|\n")
        for k in kern:
            f.write(f"| {k['name'][:60]} | {k['calls']} | {k['avg_us']:.1f} | {k['pct']:.2f} |\n")
        f.write(f"\npw:: kernels per pass: {res['pass_us']:.1f} us\n")
        f.write("achieved waves/SIMD: " + ", ".join(f"{k} {v}" for k, v in res["occupancy_waves_per_simd"].items()) + "\n")
        f.write(f"HBM bytes per pass (2*FETCH + WRITE): {res['hbm_bytes_per_launch'] / 1e6:.1f} MB "
                f"(FETCH {fetch / 1e6:.1f} MB raw, WRITE {write / 1e6:.1f} MB)\n")
        f.write("\n| kernel | reads (2*FETCH) MB | writes MB | us |\n|---|---|---|---|\n")
        us = {k["name"]: k["avg_us"] for k in kern}
        for k, c in sorted(per.items()):
            if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
                f.write(f"| {k} | {2 * c.get('FETCH_SIZE', 0) * 1024 / 1e6:.1f} | {c.get('WRITE_SIZE', 0) * 1024 / 1e6:.1f} | "
                        f"{us.get(k, 0):.1f} |\n")
        for k, c in sorted(per.items()):
            f.write(f"\n## {k} (per launch)\n\n")
            for n, v in sorted(c.items()):
                f.write(f"- {n}: {v:,.3f}\n" if (n.endswith("frac") or n.startswith("occupancy")) else f"- {n}: {v:,.1f}\n")
    print(json.dumps({k: v for k, v in res.items() if k != "pmc_per_launch"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], " ".join(sys.argv[3:]))
