#!/usr/bin/env python3
"""Counter calibration: the memory-side traffic counters of each
fetch_calib.hip pattern divided by the pattern's known bytes.

For every pattern: `requested` = the bytes the lanes ask for, `lines128` = the bytes of the
distinct 128-B lines they touch (what the L2 has to fetch at 128-B granularity).  Counter bytes:
FETCH_SIZE / WRITE_SIZE (KiB), and the request counters TCC_EA0_RDREQ_{32B,64B,128B}_sum, TCC_BUBBLE,
TCC_READ_SECTORS (32-B sectors).  The output factor `fetch_to_lines` = lines128 bytes / (FETCH_SIZE
bytes) is what a FETCH_SIZE reading of that pattern has to be multiplied by (the guide's
16-B/lane streaming factor is 2).  Usage: calibrate.py <run dir>  ->  <run dir>/calibration.{json,md}"""
import collections
import csv
import glob
import json
import os
import sys


def kname(n):
    n = n.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n.split("<")[0].strip()


def kernel_key(raw):
    """fetch_calib kernel name -> pattern name (templates carry the pattern's parameters)."""
    base = kname(raw)
    if base == "scatter":
        a = raw.split("<", 1)[1].split(">", 1)[0].replace(" ", "").split(",")
        b, line = int(a[0]), int(a[1])
        return {(4, 128): "scatter4_128", (16, 128): "scatter16_128", (4, 64): "scatter4_64",
                (16, 16): "gather16"}.get((b, line), raw)
    if base == "store16":
        return "store16_nt" if "<1>" in raw.replace(" ", "") else "store16"
    return base


def main(d):
    known = json.load(open(os.path.join(d, "known.json")))["kernels"]
    ctr = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            ctr[kernel_key(r["Kernel_Name"])][r["Counter_Name"]] = float(r["Counter_Value"])
    rows = {}
    for k, kb in known.items():
        c = ctr.get(k, {})
        fetch = c.get("FETCH_SIZE", 0.0) * 1024
        write = c.get("WRITE_SIZE", 0.0) * 1024
        req_bytes = (c.get("TCC_EA0_RDREQ_128B_sum", 0.0) * 128 + c.get("TCC_EA0_RDREQ_64B_sum", 0.0) * 64 +
                     c.get("TCC_EA0_RDREQ_32B_sum", 0.0) * 32) if "TCC_EA0_RDREQ_128B_sum" in c else None
        row = {"requested": kb["requested"], "lines128": kb["lines128"], "counters": c,
               "fetch_bytes": fetch, "write_bytes": write, "rdreq_sized_bytes": req_bytes}
        if c.get("TCC_READ_SECTORS_sum"):
            row["read_sector_bytes"] = c["TCC_READ_SECTORS_sum"] * 32
        if k.startswith("store") or k.startswith("scatter_st"):
            row["write_to_lines"] = kb["lines128"] / write if write else None
            row["write_to_requested"] = kb["requested"] / write if write else None
        else:
            row["fetch_to_lines"] = kb["lines128"] / fetch if fetch else None
            row["fetch_to_requested"] = kb["requested"] / fetch if fetch else None
            if req_bytes:
                row["sized_to_lines"] = kb["lines128"] / req_bytes
        rows[k] = row
    json.dump(rows, open(os.path.join(d, "calibration.json"), "w"), indent=1)
    with open(os.path.join(d, "calibration.md"), "w") as f:
        f.write("# Traffic-counter calibration (profiles/calib/fetch_calib.hip, 2 GiB buffer)\n\n")
        f.write("| pattern | requested MB | 128-B lines MB | FETCH MB | WRITE MB | sized RDREQ MB | sectors MB | "
                "lines / counter |\n|---|---|---|---|---|---|---|---|\n")
        for k, r in rows.items():
            fac = r.get("fetch_to_lines", r.get("write_to_lines"))
            sz = r["rdreq_sized_bytes"]
            sec = r.get("read_sector_bytes")
            f.write(f"| {k} | {r['requested'] / 1e6:.1f} | {r['lines128'] / 1e6:.1f} | {r['fetch_bytes'] / 1e6:.1f} | "
                    f"{r['write_bytes'] / 1e6:.1f} | {'' if sz is None else f'{sz / 1e6:.1f}'} | "
                    f"{'' if sec is None else f'{sec / 1e6:.1f}'} | {'' if fac is None else f'{fac:.3f}'} |\n")
    print(open(os.path.join(d, "calibration.md")).read())


if __name__ == "__main__":
    main(sys.argv[1])
