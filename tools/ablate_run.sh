#!/bin/bash
# On the GPU box: render_kernel duration and SQ counters of each tools/abl_build variant on full
# cfg2 (`pafreport -G -C`).  Usage: bash tools/ablate_run.sh <tag>
set -uo pipefail
TAG=${1:-abl}
OUT=gpurun_out/abl_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
synth/build/pwsynth paf --config 2 --fa /tmp/q2.fa --paf /tmp/a2.paf 2> /dev/null || exit 1
for d in tools/abl_build/*/; do
  v=$(basename "$d")
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/$v/tr" -o run --output-format csv -- "$d/bin/pafreport" -G -C -r /tmp/q2.fa /tmp/a2.paf -o /tmp/r_$v.txt > "$OUT/$v.log" 2>&1 || { echo "trace $v failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --kernel-include-regex "render" -d "$OUT/$v/pmc" -o run --output-format csv -- "$d/bin/pafreport" -G -C -r /tmp/q2.fa /tmp/a2.paf -o /tmp/r_$v.txt >> "$OUT/$v.log" 2>&1 || { echo "pmc $v failed"; exit 1; }
  f=$(find "$OUT/$v/tr" -name "*kernel_stats.csv" | head -1)
  us=$(grep "render_kernel" "$f" | cut -d, -f4)
  g=$(find "$OUT/$v/pmc" -name "*counter_collection.csv" | head -1)
  python3 - "$g" "$v" "$us" <<'PY'
import csv, sys, collections
t = collections.defaultdict(float)
for row in csv.DictReader(open(sys.argv[1])):
    t[row["Counter_Name"]] += float(row["Counter_Value"])
print(f"{sys.argv[2]:10s} render {float(sys.argv[3]) / 1000:8.1f} us  " + "  ".join(f"{k[3:]}={t[k] / 1e6:.1f}M" for k in sorted(t)))
PY
done
