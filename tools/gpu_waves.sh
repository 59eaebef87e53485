#!/bin/bash
# Occupancy sweep of the config-3 kernel at 65,536 documents (MT_REPLAY_WAVES), one bounded run each.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-waves}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
D=${DOCS:-65536}
for W in ${WAVES:-4 2 5}; do
  MT_REPLAY_WAVES=$W timeout -k 10 400 python -u bench.py --docs $D --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/w$W.json" 2> "$OUT/w$W.err" || { echo "w $W rc=$?"; tail "$OUT/w$W.err"; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/w$W.json')); print('waves $W', round(d['value'] / 1e6, 2), 'Mops/s', round(d['roofline']['kernel_ms'], 1), 'ms')"
done
