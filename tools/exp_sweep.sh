#!/bin/bash
# On the GPU box: kernel durations of each tools/abl_build/<variant>/lib/libpwasm_amd.so under the
# cfg2 bench (PWASM_LIB), one rocprofv3 kernel trace per variant.  Usage: tools/exp_sweep.sh <tag> [variants...]
set -uo pipefail
TAG=${1:-x}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp PW_BENCH_NOCHECK=1
VS="$*"
[ -z "$VS" ] && VS=$(ls tools/abl_build)
for v in $VS; do
  export PWASM_LIB=$PWD/tools/abl_build/$v/lib/libpwasm_amd.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sw_$TAG/$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-cfg3 --steps 10 --warmup 2 ${BENCH_ARGS:---no-gapassem} > gpurun_out/sw_${TAG}_$v.json 2> gpurun_out/sw_${TAG}_$v.err || { echo "variant $v failed: $?"; tail -5 gpurun_out/sw_${TAG}_$v.err; exit 1; }
  f=$(find gpurun_out/sw_$TAG/$v -name "*kernel_stats.csv" | head -1)
  par=$(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d.get('parity'), round(d['roofline']['kernel_ms'],4))" gpurun_out/sw_${TAG}_$v.json)
  echo "== $v parity/kernel_ms: $par"
  python3 tools/kstat.py "$f"
done
