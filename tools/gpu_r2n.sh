#!/bin/bash
# Occupancy re-sweep of the config-3 kernel after the round-2 spill changes (MT_REPLAY_WAVES=6|7|8).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2n}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for W in 6 7 8; do
  MT_REPLAY_WAVES=$W timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/w$W.json" 2> "$OUT/w$W.err" || { echo "w$W rc=$?"; tail "$OUT/w$W.err"; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/w$W.json')); print('waves $W', round(d['value'] / 1e6, 2), 'Mops/s', round(d['roofline']['kernel_ms'], 1), 'ms')"
done
