#!/bin/bash
# On the GPU box: GPU tests selected by $2, alternating sweeps of the variants ($1 rounds), then the
# 1-rank mgpu driver vs the CLI on cfg3 at scale 0.3 (phases).
# Usage: bash profiles/scripts/gpu_r6d.sh <rounds> "<pytest -k expr or ->" <tag> variant...
set -uo pipefail
R=$1; K=$2; TAG=$3; shift 3
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$K" != "-" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "$K" > gpurun_out/ab_${TAG}_pytest.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/ab_${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_${TAG}_pytest.log
fi
for i in $(seq 1 $R); do
  bash tools/exp_sweep.sh ${TAG}_$i "$@" || exit 1
done
D=$(mktemp -d /tmp/c3XXXX)
./synth/build/pwsynth paf --config 3 --scale 0.3 --seed 3 --fa $D/q.fa --paf $D/a.paf --threads 16 2>/dev/null || exit 1
PW_PROFILE_HOST=1 timeout -k 10 200 ./pwasm_amd/bin/pafreport -G -C -r $D/q.fa $D/a.paf -o $D/cli.txt 2> gpurun_out/cli3_$TAG.err || { echo "cli failed"; exit 1; }
grep "\[cli\] total\|cli-dev" gpurun_out/cli3_$TAG.err
S=$(date +%s%N)
PW_PROFILE_HOST=1 timeout -k 10 300 python3 -m pwasm_amd.mgpu -G -C -r $D/q.fa $D/a.paf -o $D/mg.txt 2> gpurun_out/mg3_$TAG.err || { echo "mgpu failed"; tail gpurun_out/mg3_$TAG.err; exit 1; }
E=$(date +%s%N)
echo "mgpu wall $(( (E - S) / 1000000 )) ms"
grep "mgpu" gpurun_out/mg3_$TAG.err
cmp $D/cli.txt $D/mg.txt && echo "same bytes"
rm -rf $D
