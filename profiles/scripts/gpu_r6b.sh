#!/bin/bash
# On the GPU box: counter calibration, then the 1-rank mgpu driver vs the CLI on cfg3 at scale $1 (phases).
set -uo pipefail
SC=${1:-0.3}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash profiles/calib/run_calib.sh r6 > gpurun_out/calib_r6.log 2>&1 || { echo "calib failed"; tail -20 gpurun_out/calib_r6.log; }
tail -16 gpurun_out/calib_r6.log
D=$(mktemp -d /tmp/c3XXXX)
./synth/build/pwsynth paf --config 3 --scale $SC --seed 3 --fa $D/q.fa --paf $D/a.paf --threads 16 2>/dev/null || exit 1
ls -la $D
T0=$(date +%s.%N)
PW_PROFILE_HOST=1 timeout -k 10 200 ./pwasm_amd/bin/pafreport -G -C -r $D/q.fa $D/a.paf -o $D/cli.txt 2> gpurun_out/cli3.err || { echo "cli failed"; exit 1; }
T1=$(date +%s.%N)
echo "cli wall $(echo "$T1 - $T0" | bc)"
grep "\[cli\]" gpurun_out/cli3.err | tail -8
T0=$(date +%s.%N)
PW_PROFILE_HOST=1 timeout -k 10 300 python3 -m pwasm_amd.mgpu -G -C -r $D/q.fa $D/a.paf -o $D/mg.txt 2> gpurun_out/mg3.err || { echo "mgpu failed"; tail gpurun_out/mg3.err; exit 1; }
T1=$(date +%s.%N)
echo "mgpu wall $(echo "$T1 - $T0" | bc)"
grep "mgpu" gpurun_out/mg3.err
cmp $D/cli.txt $D/mg.txt && echo "same bytes"
rm -rf $D
