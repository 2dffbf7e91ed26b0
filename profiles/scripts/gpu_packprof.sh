#!/bin/bash
# On the GPU box: the cs packer alone (tools/exp_packtime.py) — its time, then a kernel trace and
# two PMC passes restricted to pack_cs_kernel.
set -uo pipefail
TAG=${1:-pk}
O=gpurun_out/packprof_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/exp_packtime.py > $O/time.txt 2>&1 || { echo "packtime failed"; tail $O/time.txt; exit 1; }
cat $O/time.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/exp_packtime.py > /dev/null 2> $O/trace.err || { echo "trace failed"; exit 1; }
python3 tools/kstats.py $O/trace/run_kernel_stats.csv
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "pack_cs" -d $O/pmc_$i -o run --output-format csv -- python3 tools/exp_packtime.py > /dev/null 2> $O/pmc_$i.err || { echo "pmc $i failed"; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "pack_cs" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
disp = {}
for k in tot:
    disp[k] = tot[k]
print({k: round(v) for k, v in sorted(disp.items())})
PY
echo packprof done
