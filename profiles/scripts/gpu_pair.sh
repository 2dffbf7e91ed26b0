#!/bin/bash
# On the GPU box: parity of the two-records-per-wave index kernel, then cfg3 (scale 0.2) kernel
# traces with and without it.  Usage: profiles/scripts/gpu_pair.sh <tag>
set -uo pipefail
TAG=${1:-pair}
mkdir -p gpurun_out/pair_$TAG
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gapassem_refine.py tests/test_gapassem_kat.py tests/test_gapassem_shard.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gapassem or refine or msa or pair or cfg3 or kat or edge_mix or error_midway or cfg2 or long" > gpurun_out/pair_$TAG/pytest.log 2>&1 || { echo "pytest failed: $?"; grep -E "FAIL|Error|error|first difference|oracle:|hip:" gpurun_out/pair_$TAG/pytest.log | head -30; tail -5 gpurun_out/pair_$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/pair_$TAG/pytest.log
for mode in pairs single; do
  if [ $mode = single ]; then export PW_NO_PAIRS=1; else unset PW_NO_PAIRS; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pair_$TAG/$mode -o run --output-format csv -- python3 bench.py --config 3 --scale 0.2 --steps 5 --warmup 1 --no-parity --no-cpu-baseline > gpurun_out/pair_$TAG/$mode.json 2> gpurun_out/pair_$TAG/$mode.err || { echo "bench $mode failed"; tail -5 gpurun_out/pair_$TAG/$mode.err; exit 1; }
  echo "== $mode kernel_ms $(python3 -c "import json;print(json.load(open('gpurun_out/pair_$TAG/$mode.json'))['roofline']['kernel_ms'])")"
  python3 tools/kstat.py $(find gpurun_out/pair_$TAG/$mode -name "*kernel_stats.csv" | head -1)
done
