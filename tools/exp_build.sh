#!/bin/bash
# Build timing-only ablation variants of libpwasm_amd.so into build_exp/ (never shipped):
#   [EXP_TAG=t] [EXP_FLAGS=-D...] bash tools/exp_build.sh 1 2 4 ...
#      -> build_exp/libpwasm_amd_<tag><n>.so  (-DPW_ABL=<n> $EXP_FLAGS)
# Run one with PWASM_LIB=build_exp/libpwasm_amd_<tag><n>.so python bench.py ...
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p build_exp
T=${EXP_TAG:-}
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Ipwasm_amd/csrc ${EXP_FLAGS:-}"
for n in "$@"; do
  /opt/rocm/bin/hipcc $F -DPW_ABL=$n -c pwasm_amd/csrc/pw_report.hip -o build_exp/pw_report_$T$n.o &
done
wait
for n in "$@"; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build_exp/libpwasm_amd_$T$n.so build_exp/pw_report_$T$n.o \
    pwasm_amd/build/pw_host.o pwasm_amd/build/pw_msa.o pwasm_amd/build/pw_gapassem.o
done
