#!/bin/bash
# On the GPU box: per-kernel SQ counters of the CLI on event-type-specific inputs (see exp_mix.sh).
# Usage: MIXES="name:args_with_underscores ..." bash tools/exp_mix_pmc.sh <tag>
set -uo pipefail
TAG=${1:-mixp}
OUT=gpurun_out/mixp_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in ${MIXES:-"def:"}; do
  name=${m%%:*}; args=${m#*:}; args=${args//_/ }
  synth/build/pwsynth paf --config 2 --fa /tmp/q_$name.fa --paf /tmp/a_$name.paf $args 2> /dev/null || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_BRANCH --kernel-include-regex "render" -d "$OUT/$name" -o run --output-format csv -- pwasm_amd/bin/pafreport -G -C -r /tmp/q_$name.fa /tmp/a_$name.paf -o /tmp/r_$name.txt > "$OUT/$name.log" 2>&1 || { echo "pmc $name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "== $name"
  f=$(find "$OUT/$name" -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
t = collections.defaultdict(float)
for row in csv.DictReader(open(sys.argv[1])):
    t[row["Counter_Name"]] += float(row["Counter_Value"])
for k in sorted(t): print(f"  {k:24s} {t[k]:>16,.0f}")
PY
done
