set -uo pipefail
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "outfile or output_file or many_batches or kat or cfg2_sub or emit" > gpurun_out/pytest_emit.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_emit.log; exit 1; }
tail -2 gpurun_out/pytest_emit.log
bash profiles/scripts/gpu_e2e3.sh e3c
