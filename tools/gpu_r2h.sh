#!/bin/bash
# Forced vs compiler-chosen inlining (distinct kernels now) at 65,536 docs, 8 waves; then the
# memory-pipeline counters (tools/gpu_mem.sh).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for NI in 1 0; do
  MT_REPLAY_NOINLINE=$NI MT_REPLAY_WAVES=8 timeout -k 10 400 python -u bench.py --docs 65536 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/ni${NI}.json" 2> "$OUT/ni${NI}.err" || { echo "ni $NI rc=$?"; tail "$OUT/ni${NI}.err"; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/ni${NI}.json')); print('noinline $NI waves 8', round(d['value'] / 1e6, 2), 'Mops/s', round(d['roofline']['kernel_ms'], 1), 'ms')"
done
bash tools/gpu_mem.sh $TAG/mem
