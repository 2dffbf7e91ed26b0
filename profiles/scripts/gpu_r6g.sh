#!/bin/bash
# On the GPU box: the HIP runtime's start-up, five runs each default / ROCR_VISIBLE_DEVICES=0.
set -uo pipefail
B=profiles/calib/hip_init
[ -x $B ] || /opt/rocm/bin/hipcc -O2 profiles/calib/hip_init.cpp -o $B || exit 1
echo "ROCR_VISIBLE_DEVICES=${ROCR_VISIBLE_DEVICES:-unset} HIP_VISIBLE_DEVICES=${HIP_VISIBLE_DEVICES:-unset}"
ls /dev/dri 2>/dev/null | tr '\n' ' '; echo; ls /sys/class/kfd/kfd/topology/nodes 2>/dev/null | wc -l
for i in 1 2 3 4 5; do timeout -k 5 60 $B || exit 1; done
for i in 1 2 3; do ROCR_VISIBLE_DEVICES=0 timeout -k 5 60 $B || exit 1; done
for i in 1 2 3; do HSA_ENABLE_SDMA=0 timeout -k 5 60 $B || exit 1; done
