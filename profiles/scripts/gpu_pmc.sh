#!/bin/bash
# On the GPU box: PMC passes (one counter group per run) for the kernels matching a regex.
# Usage: profiles/scripts/gpu_pmc.sh <tag> <kernel regex> [bench args...]
set -uo pipefail
TAG=${1:-p}; KR=${2:-render_kernel}; shift 2
mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
B="bench.py --no-cpu-baseline --no-parity --steps 4 --warmup 1 $*"
i=0
for G in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -k 5 120 rocprofv3 --pmc $G --kernel-include-regex "$KR" -d gpurun_out/pmc_$TAG/p$i -o run --output-format csv -- python3 $B > /dev/null 2> gpurun_out/pmc_$TAG/p$i.err || { echo "pmc pass $i failed: $?"; tail -5 gpurun_out/pmc_$TAG/p$i.err; exit 1; }
done
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/pmc_{tag}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:40s} {c:24s} {sum(v)/len(v):18,.1f}")
PY
