#!/bin/bash
# Every GPU test, then the config-5 and config-4 lines (heap sift-down with 5-level lookahead, staged
# window pass, parallel leaf search).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|ERROR|Error" "$OUT/pytest_gpu.txt" | head -20; tail -5 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
for C in 5 4; do
  timeout -k 10 900 python -u bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c$C.json" 2> "$OUT/c$C.err" || { echo "c$C rc=$?"; tail -20 "$OUT/c$C.err"; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/c$C.json')); print('config $C', round(d['value'] / 1e6, 2), 'Mops/s', round(d['roofline']['kernel_ms'], 1), 'ms')"
done
