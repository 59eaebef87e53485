#!/bin/bash
# GPU tests, the default (config-3) bench line and its rocprofv3 kernel-trace summary (CSV).
# Every GPU step is bounded and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
# a heartbeat under gpurun_out/ while long steps run (each step has its own time limit)
( while sleep 60; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|ERROR|Error" "$OUT/pytest_gpu.txt" | head -20; tail -5 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
[ -n "$TESTS_ONLY" ] && exit 0
timeout -k 10 400 python -u bench.py $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo "trace rc=$?"; tail -20 "$OUT/trace.err"; exit 1; }
find "$OUT/trace" -name '*kernel_stats.csv' -exec head -3 {} \;
