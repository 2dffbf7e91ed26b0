#!/bin/bash
# Local: copy the judged parts of a profile run (gpurun_out/prof_<tag>) into profiles/<name>.
# Usage: tools/save_prof.sh <tag> <name> [extra files from gpurun_out ...]
set -euo pipefail
S=gpurun_out/prof_$1; D=profiles/$2; shift 2
mkdir -p "$D"
cp "$S/summary.md" "$S/summary.json" "$D/"
cp "$S/trace/run_kernel_stats.csv" "$D/kernel_stats.csv"
for f in "$@"; do cp "gpurun_out/$f" "$D/"; done
ls "$D"
