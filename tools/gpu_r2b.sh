#!/bin/bash
# Round-2: GPU tests (incl. config-4 tiled parity) + a config-4 bench at 1/10 of the ops (per-op cost).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2b}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -3 "$OUT/pytest_gpu.txt"
timeout -k 10 600 python -u bench.py --config 4 --ops-per-doc 100000 --steps 1 --warmup 0 > "$OUT/bench_c4_100k.json" 2> "$OUT/bench_c4_100k.err" || { echo "bench c4 failed rc=$?"; tail -20 "$OUT/bench_c4_100k.err"; exit 1; }
cat "$OUT/bench_c4_100k.json"
