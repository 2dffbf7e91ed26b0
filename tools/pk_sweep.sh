#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in cur pk_buf cur pk_buf; do
  PWASM_LIB=$PWD/tools/abl_build/$v/lib/libpwasm_amd.so timeout -k 10 200 python3 tools/pack_bench.py 20 > gpurun_out/pk_$v.json 2> gpurun_out/pk_$v.err || { echo "failed $v"; tail -5 gpurun_out/pk_$v.err; exit 1; }
  echo "$v $(cat gpurun_out/pk_$v.json)"
done
