#!/bin/bash
# Profile recipe (run on the MI355X box from the repo root): bench, kernel trace + stats, and
# separate PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
# Usage: bash profiles/run_prof.sh <tag>
set -euo pipefail
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $B > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex report_kernel -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 $B > /dev/null 2> "$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex report_kernel -d "$OUT/pmc_write" -o run --output-format csv -- python3 $B > /dev/null 2> "$OUT/pmc_write.err"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex report_kernel -d "$OUT/pmc_sq" -o run --output-format csv -- python3 $B > /dev/null 2> "$OUT/pmc_sq.err"
# stall / instruction-mix passes (SQ_* cycle counters are in quad-cycles)
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS --kernel-include-regex report_kernel -d "$OUT/pmc_stall" -o run --output-format csv -- python3 $B > /dev/null 2> "$OUT/pmc_stall.err"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM --kernel-include-regex report_kernel -d "$OUT/pmc_insts" -o run --output-format csv -- python3 $B > /dev/null 2> "$OUT/pmc_insts.err"
echo "profile done: $OUT"
