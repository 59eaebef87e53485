#!/bin/bash
# GPU tests, then config 4 (one step, with its CPU-baseline sample of 16 full-size documents). Bounded; stops
# at the first failure. usage: tools/gpu_c4.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-c4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
( while sleep 60; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|ERROR|Error" "$OUT/pytest_gpu.txt" | head -20; tail -5 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 900 python -u bench.py --config 4 --steps 1 --warmup 1 > "$OUT/c4.json" 2> "$OUT/c4.err" || { echo "c4 rc=$?"; tail "$OUT/c4.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/c4.json'));print('c4', round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],1), d['roofline']['frac'], d['cpu_baseline']['sample'])"
