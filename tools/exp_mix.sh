#!/bin/bash
# On the GPU box: render/index kernel time per event for event-type mixes (cfg2 shape, 100k
# records): default, indels only, substitutions only.  Usage: bash tools/exp_mix.sh <tag>
set -uo pipefail
TAG=${1:-mix}
OUT=gpurun_out/mix_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in ${MIXES:-"def:" "indel:--psub 0" "sub:--psub 1 --pdel 0 --pins 0"}; do
  name=${m%%:*}; args=${m#*:}; args=${args//_/ }
  synth/build/pwsynth paf --config 2 --fa /tmp/q_$name.fa --paf /tmp/a_$name.paf $args 2> /dev/null || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv -- pwasm_amd/bin/pafreport -G -C -r /tmp/q_$name.fa /tmp/a_$name.paf -o /tmp/r_$name.txt > "$OUT/$name.log" 2>&1 || { echo "run $name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  ev=$(grep -c -v '^>' /tmp/r_$name.txt)
  echo "== $name events=$ev"
  f=$(find "$OUT/$name" -name "*kernel_stats.csv" | head -1)
  grep "pw::" "$f" | cut -d, -f1,2,4 | sed 's/(pw_report_args, pw::Work)//'
done
