#!/bin/bash
# Round-2 re-entry check: GPU tests, the default config-3 line with its kernel-trace summary, then
# the config-4 and config-5 lines. Each GPU step is bounded; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpu_round.sh $TAG || exit 1
for C in 5 4; do
  timeout -k 10 900 python -u bench.py --config $C --steps 2 --warmup 1 > "$OUT/c$C.json" 2> "$OUT/c$C.err" || { echo "c$C rc=$?"; tail -20 "$OUT/c$C.err"; exit 1; }
  cat "$OUT/c$C.json"
done
