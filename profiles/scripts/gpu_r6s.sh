#!/bin/bash
# On the GPU box: render_kernel read-stream attribution.  Per variant of tools/abl_build (one
# render input stream pointed at a fixed, L2-resident address: timing / traffic only), a kernel
# trace and a FETCH_SIZE pass (cfg2 bench, 10 steps), then the per-kernel mean duration and
# FETCH_SIZE (x2: profiles/r6_calib) per dispatch.  Usage: bash profiles/scripts/gpu_r6s.sh <tag> variant...
set -uo pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp PW_BENCH_NOCHECK=1
B="bench.py --no-cpu-baseline --no-cfg3 --no-gapassem --no-parity --no-e2e --steps 10 --warmup 2"
for v in "$@"; do
  export PWASM_LIB=$PWD/tools/abl_build/$v/lib/libpwasm_amd.so
  O=gpurun_out/st_$TAG/$v
  mkdir -p $O
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O.trace.json 2> $O.trace.err || { echo "trace $v failed"; tail -5 $O.trace.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "pw::" -d $O/pmc -o run --output-format csv -- python3 $B > /dev/null 2> $O.pmc.err || { echo "pmc $v failed"; tail -5 $O.pmc.err; exit 1; }
  python3 - "$O" "$v" <<'PY'
import csv, glob, sys, collections
o, v = sys.argv[1], sys.argv[2]
dur = collections.defaultdict(list)
for f in glob.glob(f"{o}/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
pmc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{o}/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        pmc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(dur):
    if not k.startswith("pw::"):
        continue
    d = sorted(dur[k])[len(dur[k]) // 2]
    fs = pmc[k].get("FETCH_SIZE", [0])
    print(f"{v:8s} {k[:34]:34s} median {d:8.1f} us  read {2 * sum(fs) / len(fs) / 1e3:8.1f} MB")
PY
done
