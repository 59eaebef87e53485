#!/bin/bash
# Round-2: full GPU test tier, the default (config-3) bench line, and its rocprofv3 kernel summary.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2d}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR" "$OUT/pytest_gpu.txt" | head -20; tail -2 "$OUT/pytest_gpu.txt"
[ $rc -le 1 ] || exit 1
timeout -k 10 600 python -u bench.py > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || { echo "bench failed rc=$?"; tail -20 "$OUT/bench_c3.err"; exit 1; }
cat "$OUT/bench_c3.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o c3 -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_c3_prof.json" 2> "$OUT/bench_c3_prof.err" || { echo "rocprof failed rc=$?"; tail -20 "$OUT/bench_c3_prof.err"; exit 1; }
find "$OUT/prof_c3" -name "*stats*" | head
