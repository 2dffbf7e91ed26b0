#!/bin/bash
# On the GPU box: pack_cs_kernel alone (tools/pack_bench.py) — timing + parity, a kernel trace and
# PMC passes.  Usage: profiles/scripts/gpu_pack.sh <tag>
set -uo pipefail
TAG=${1:-pk}
O=gpurun_out/pack_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/pack_bench.py 20 > $O/run.json 2> $O/run.err || { echo "pack run failed"; tail -5 $O/run.err; exit 1; }
cat $O/run.json
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT" \
         "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 5 120 rocprofv3 --pmc $G --kernel-include-regex "pw::pack_cs" -d $O/pmc_$i -o run --output-format csv -- python3 tools/pack_bench.py 5 > /dev/null 2> $O/pmc_$i.err || { echo "pmc pass $i failed"; tail -5 $O/pmc_$i.err; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(d.items()):
    c = {n: sum(v) / len(v) for n, v in cs.items()}
    print(k)
    for n in sorted(c):
        print(f"   {n:34s} {c[n]:16,.0f}")
PY
