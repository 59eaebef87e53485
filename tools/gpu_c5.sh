#!/bin/bash
# GPU parity tests, then the config-5 bench (PermutationVector replicas) and its kernel summary.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-c5}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -3 "$OUT/pytest_gpu.txt"
timeout -k 10 600 python -u bench.py --config 5 --steps 2 --warmup 1 --cpu-sample-docs 2048 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { echo "bench c5 rc=$?"; tail -20 "$OUT/bench_c5.err"; exit 1; }
cat "$OUT/bench_c5.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/trace_c5.json" 2> "$OUT/trace_c5.err" || { echo "trace rc=$?"; tail -20 "$OUT/trace_c5.err"; exit 1; }
find "$OUT/trace" -name '*kernel_stats.csv' -exec cat {} \;
