#!/bin/bash
# On the GPU box: tile_counts attribution (tools/exp_msa_variants.py builds): per variant a kernel
# trace of the cfg5 bench and one PMC pass of the LDS counters.  Usage: profiles/scripts/gpu_msa_attr.sh <tag> [variants]
set -uo pipefail
TAG=${1:-ma}; shift
VS="${*:-cur noflush nowin noruns rp_lds}"
mkdir -p gpurun_out
export TMPDIR=/tmp PW_BENCH_NOCHECK=1
for v in $VS; do
  export PWASM_LIB=$PWD/tools/abl_build/$v/lib/libpwasm_amd.so
  O=gpurun_out/ma_$TAG/$v
  mkdir -p $O
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --config 5 --no-parity --no-cpu-baseline --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo "variant $v trace failed: $?"; tail -5 $O/bench.err; exit 1; }
  timeout -k 5 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --kernel-include-regex "pw::" -d $O/pmc -o run --output-format csv -- python3 bench.py --config 5 --no-parity --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2> $O/pmc.err || { echo "variant $v pmc failed: $?"; tail -5 $O/pmc.err; exit 1; }
  echo "== $v"
  f=$(find $O/trace -name "*kernel_stats.csv" | head -1)
  python3 tools/kstat.py "$f"
done
