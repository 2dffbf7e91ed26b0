#!/bin/bash
# On the GPU box: tools/pack_bench.py (the cs packer alone on cfg2) per variant build.
# Usage: tools/pk_sweep.sh [variants...]
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VS="${*:-cur pk_buf cur pk_buf}"
for v in $VS; do
  PWASM_LIB=$PWD/tools/abl_build/$v/lib/libpwasm_amd.so timeout -k 10 200 python3 tools/pack_bench.py 20 > gpurun_out/pk_$v.json 2> gpurun_out/pk_$v.err || { echo "failed $v"; tail -5 gpurun_out/pk_$v.err; exit 1; }
  echo "$v $(cat gpurun_out/pk_$v.json)"
done
