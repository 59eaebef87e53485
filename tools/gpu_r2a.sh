#!/bin/bash
# Round-2 check: GPU tests on the product build and on the no-compiler-barrier build, then short
# benches of configs 1, 2 and a 16k-doc config 3. Each GPU step is bounded; stop at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2a}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu.txt"
MT_REPLAY_LIB=fluidframework_amd/build/libmtreplay_noclob.so timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_noclob.txt" 2>&1 || { echo "noclob pytest failed rc=$?"; tail -30 "$OUT/pytest_gpu_noclob.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu_noclob.txt"
for C in 1 2; do
  timeout -k 10 300 python -u bench.py --config $C --steps 3 --warmup 1 > "$OUT/bench_c$C.json" 2> "$OUT/bench_c$C.err" || { echo "bench c$C failed rc=$?"; tail -20 "$OUT/bench_c$C.err"; exit 1; }
  cat "$OUT/bench_c$C.json"
done
timeout -k 10 300 python -u bench.py --docs 16384 --steps 3 --warmup 1 > "$OUT/bench_c3_16k.json" 2> "$OUT/bench_c3_16k.err" || { echo "bench c3 failed rc=$?"; tail -20 "$OUT/bench_c3_16k.err"; exit 1; }
cat "$OUT/bench_c3_16k.json"
