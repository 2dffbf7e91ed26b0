#!/bin/bash
# On the GPU box: the counter calibration (fetch_calib.hip), one rocprofv3 --pmc pass per
# counter group, then calibrate.py.  Usage: bash profiles/calib/run_calib.sh <tag>
set -uo pipefail
TAG=${1:-calib}
OUT=gpurun_out/calib_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B=profiles/calib/fetch_calib
[ -x $B ] || /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 profiles/calib/fetch_calib.hip -o $B || exit 1
timeout -k 10 120 $B > "$OUT/known.json" || { echo "calib run failed"; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $B > /dev/null 2> "$OUT/trace.err" || { echo "trace failed"; tail -5 "$OUT/trace.err"; exit 1; }
i=0
for G in "FETCH_SIZE" "WRITE_SIZE" \
         "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
         "TCC_BUBBLE_sum TCC_READ_SECTORS_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum" \
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WR_UNCACHED_32B_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $G -d "$OUT/pmc_$i" -o run --output-format csv -- $B > /dev/null 2> "$OUT/pmc_$i.err" || { echo "pmc pass $i ($G) failed: $?"; tail -3 "$OUT/pmc_$i.err"; }
done
python3 profiles/calib/calibrate.py "$OUT" && echo "calibration done: $OUT"
