#!/bin/bash
# Round-2 closing check: every GPU test (incl. delta events, local references, reconnect), the default
# config-3 line with cpu_baseline and its kernel-trace summary, then the config-2 and config-1 lines.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2l}
OUT=gpurun_out/$TAG
bash tools/gpu_round.sh $TAG || exit 1
for C in 2 1; do
  timeout -k 10 600 python -u bench.py --config $C --steps 2 --warmup 1 > "$OUT/c$C.json" 2> "$OUT/c$C.err" || { echo "c$C rc=$?"; tail -20 "$OUT/c$C.err"; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/c$C.json')); print('config $C', round(d['value'] / 1e6, 2), 'Mops/s', round(d['roofline']['kernel_ms'], 1), 'ms')"
done
