#!/bin/bash
# On the GPU box: for each experiment build, one PMC pass (instruction mix of one kernel) + timing.
# Usage: tools/gpu_abl_pmc.sh <kernel regex> <tag> <tag> ...   (build_exp/libpwasm_amd_<tag>.so)
set -uo pipefail
KR=$1; shift
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY"
for t in "$@"; do
  PWASM_LIB=$PWD/build_exp/libpwasm_amd_$t.so timeout -k 5 120 rocprofv3 --pmc $C --kernel-include-regex "$KR" -d gpurun_out/abl/$t -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/abl/$t.json 2> gpurun_out/abl/$t.err || { echo "pmc $t failed: $?"; tail -5 gpurun_out/abl/$t.err; exit 1; }
  PWASM_LIB=$PWD/build_exp/libpwasm_amd_$t.so timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 20 > gpurun_out/abl/$t.t.json 2>/dev/null || { echo "bench $t failed"; exit 1; }
done
python3 - "$@" <<'PY'
import csv, glob, json, sys, collections
for t in sys.argv[1:]:
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/abl/{t}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in acc.items()}
    ms = json.load(open(f"gpurun_out/abl/{t}.t.json"))["roofline"]["kernel_ms"]
    print(f"{t:10s} ms={ms:.4f} " + " ".join(f"{k.replace('SQ_INSTS_','').replace('SQ_','')}={v/1e6:.2f}M" for k, v in sorted(m.items())))
PY
