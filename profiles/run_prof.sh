#!/bin/bash
# Profile recipe (run on the MI355X box from the repo root): kernel trace + stats of the bench,
# then separate PMC passes (one counter group per run: FETCH_SIZE and WRITE_SIZE cannot share
# a pass on gfx950), all restricted to the pw:: kernels, then the summary.
# Usage: bash profiles/run_prof.sh <tag> [extra bench args]
set -uo pipefail
TAG=${1:-r1}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-gapassem --no-cfg3 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $B > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || { echo "trace failed"; exit 1; }
i=0
for G in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA" \
         "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 5 120 rocprofv3 --pmc $G --kernel-include-regex "pw::" -d "$OUT/pmc_$i" -o run --output-format csv -- python3 $B > /dev/null 2> "$OUT/pmc_$i.err" || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc_$i.err"; exit 1; }
done
python3 profiles/summarize.py "$OUT" "$OUT/summary" $* && echo "profile done: $OUT"
