#!/bin/bash
# On the GPU box (round 5): cache-policy A/B sweeps of the report, GapAssem and packer kernels.
set -uo pipefail
mkdir -p gpurun_out
BENCH_ARGS=--no-gapassem bash profiles/scripts/gpu_ab.sh pol "report or kat or cli or long" 2 cur hot_nt tx_nt ops_nt || exit 1
bash profiles/scripts/gpu_msa_attr.sh polm cur ofs_nt seq_nt cur ofs_nt seq_nt || exit 1
bash tools/pk_sweep.sh cur pk_nt cur pk_nt || exit 1
