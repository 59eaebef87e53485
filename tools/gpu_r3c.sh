#!/bin/bash
# Targeted GPU tests of the promotion / legacy-summary work (every step bounded, stops at a failure).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3c
mkdir -p "$OUT"
( while sleep 60; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_caps.py tests/test_legacy_ref.py tests/test_annotate_kat.py tests/test_golden_snapshots.py -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|ERROR|Error|assert" "$OUT/pytest_gpu.txt" | head -30; tail -5 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
