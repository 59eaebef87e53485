#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2c}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/gpu_tiled_dbg.py > "$OUT/tiled_dbg.txt" 2>&1 || { echo "dbg failed rc=$?"; tail -20 "$OUT/tiled_dbg.txt"; exit 1; }
cat "$OUT/tiled_dbg.txt"
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1; echo "pytest rc=$?"
grep -E "PASSED|FAILED|ERROR" "$OUT/pytest_gpu.txt" | grep -v PASSED | head -20; tail -2 "$OUT/pytest_gpu.txt"
timeout -k 10 600 python -u bench.py --config 4 --ops-per-doc 100000 --steps 1 --warmup 0 > "$OUT/bench_c4_100k.json" 2> "$OUT/bench_c4_100k.err" || { echo "bench c4 failed rc=$?"; tail -20 "$OUT/bench_c4_100k.err"; exit 1; }
cat "$OUT/bench_c4_100k.json"
