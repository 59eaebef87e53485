#!/bin/bash
# Delta-event build: every GPU test (incl. tests/test_ref_deltas.py) and a short default bench (the hot
# kernel is built without delta emission; its rate must not move).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2j}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|ERROR|Error" "$OUT/pytest_gpu.txt" | head -20; tail -5 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
