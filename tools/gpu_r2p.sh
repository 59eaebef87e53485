#!/bin/bash
# GPU tests, then the config-3 line for the in-tree library and two register-allocation variants of
# the replay core built from scratch copies (A: root / nfree / hwHeap / seqOps out of the register
# header; C: A + freeHead / nfreeRid), each with its own library (MT_REPLAY_LIB).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2p}
OUT=gpurun_out/$TAG
TESTS_ONLY=1 bash tools/gpu_round.sh $TAG || exit 1
for V in base a c; do
  L=fluidframework_amd/build/libmtreplay.so
  [ "$V" != base ] && L=fluidframework_amd/build/libmtreplay_$V.so
  MT_REPLAY_LIB=$L timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/$V.json" 2> "$OUT/$V.err" || { echo "$V rc=$?"; tail "$OUT/$V.err"; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/$V.json')); print('$V', round(d['value'] / 1e6, 2), 'Mops/s', round(d['roofline']['kernel_ms'], 1), 'ms')"
done
