#!/bin/bash
# Round-2: GPU tests, then the config-3 bench line + kernel trace + HBM traffic counters.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2e}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR" "$OUT/pytest_gpu.txt" | head -20; tail -2 "$OUT/pytest_gpu.txt"
[ $rc -le 1 ] || exit 1
PMC=1 bash tools/gpu_bench.sh "${1:-r2e}/c3" || exit 1
