#!/bin/bash
# GPU tests, then the default config-3 bench and its kernel trace (bounded; stops at the first failure).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r3g}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
( while sleep 60; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|ERROR|Error" "$OUT/pytest_gpu.txt" | head -20; tail -5 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 600 python -u bench.py --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err" || { echo "bench rc=$?"; tail -20 "$OUT/c3.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/c3.json'));print('c3', round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],1), d['roofline']['frac'])"
[ -n "$MORE" ] && { timeout -k 10 400 python -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c2.json" 2> "$OUT/c2.err" || exit 1; python -c "import json;d=json.load(open('$OUT/c2.json'));print('c2', round(d['value']/1e6,2))"; }
exit 0
