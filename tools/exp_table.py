"""Local: per-launch kernel averages of an exp_sweep.sh run (gpurun_out/sw_<tag>/<variant>)."""
import csv
import glob
import json
import os
import sys

tag = sys.argv[1]
base = f"gpurun_out/sw_{tag}"
ks = sys.argv[2].split(",") if len(sys.argv) > 2 else ["index", "tctx", "render", "fixup", "stop_table"]
print(f"{'variant':16s} " + " ".join(f"{k:>10s}" for k in ks) + "   kernel_ms parity")
for v in sorted(os.listdir(base)):
    f = glob.glob(f"{base}/{v}/**/*kernel_stats.csv", recursive=True)
    if not f:
        continue
    avg = {}
    for row in csv.DictReader(open(f[0])):
        for k in ks:
            if row["Name"].startswith(f"pw::{k}_kernel") or row["Name"].startswith(f"pw::{k}("):
                avg[k] = float(row["AverageNs"]) / 1000
    try:
        j = json.load(open(f"gpurun_out/sw_{tag}_{v}.json"))
        km, par = j["roofline"]["kernel_ms"], j.get("parity")
    except Exception:
        km, par = float("nan"), "?"
    print(f"{v:16s} " + " ".join(f"{avg.get(k, 0):10.1f}" for k in ks) + f"   {km:.4f} {par}")
