#!/bin/bash
# On the GPU box: PMC passes (one group per run) over the cfg2 bench for the report kernels, then a
# per-kernel table.  Usage: profiles/scripts/gpu_rpmc.sh <tag> [kernel regex]
set -uo pipefail
TAG=${1:-rp}
RX=${2:-"pw::(render|index|tctx)_kernel"}
O=gpurun_out/rpmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-gapassem ${BENCH_ARGS:-}"
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
         "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL" \
         "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 5 120 rocprofv3 --pmc $G --kernel-include-regex "$RX" -d $O/pmc_$i -o run --output-format csv -- python3 $B > /dev/null 2> $O/pmc_$i.err || { echo "pmc pass $i failed"; tail -5 $O/pmc_$i.err; exit 1; }
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
        print(f"   {n:24s} {c[n]:16,.0f}")
PY
