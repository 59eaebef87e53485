#!/bin/bash
# GPU tests, config 3 (with its kernel trace), configs 2 and 5, and config 4 with its CPU-baseline sample
# (16 full-size documents through the oracle). Bounded; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r3h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
( while sleep 60; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|ERROR|Error" "$OUT/pytest_gpu.txt" | head -20; tail -5 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 600 python -u bench.py > "$OUT/c3.json" 2> "$OUT/c3.err" || { echo "bench rc=$?"; tail -20 "$OUT/c3.err"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo "trace rc=$?"; tail -20 "$OUT/trace.err"; exit 1; }
timeout -k 10 400 python -u bench.py --config 2 --steps 3 --warmup 1 > "$OUT/c2.json" 2> "$OUT/c2.err" || { echo "c2 rc=$?"; tail "$OUT/c2.err"; exit 1; }
timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err" || { echo "c5 rc=$?"; tail "$OUT/c5.err"; exit 1; }
for f in c3 c2 c5; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f', round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],1), d['roofline']['frac'])"; done
timeout -k 10 900 python -u bench.py --config 4 --steps 1 --warmup 1 > "$OUT/c4.json" 2> "$OUT/c4.err" || { echo "c4 rc=$?"; tail "$OUT/c4.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/c4.json'));print('c4', round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],1), d['roofline']['frac'], d['cpu_baseline'])"
