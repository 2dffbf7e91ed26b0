#!/bin/bash
# On the GPU box: where the CLI's wall clock goes on full cfg2 (PW_PROFILE_HOST phase timings).
set -uo pipefail
mkdir -p gpurun_out
synth/build/pwsynth paf --config 2 --fa /tmp/q2.fa --paf /tmp/a2.paf 2> /dev/null || exit 1
for i in 1 2; do  # (no time(1) on the box: python timing)
  python3 -c "import subprocess,time; t=time.time(); subprocess.run([\"pwasm_amd/bin/pafreport\",\"-G\",\"-C\",\"-r\",\"/tmp/q2.fa\",\"/tmp/a2.paf\",\"-o\",\"/tmp/r2.txt\"]); print(\"cli wall\", round(time.time()-t,3))"
done
PW_PROFILE_HOST=1 timeout -k 10 120 pwasm_amd/bin/pafreport -G -C -r /tmp/q2.fa /tmp/a2.paf -o /tmp/r2.txt 2>&1 | tail -20
