#!/bin/bash
# Forced vs compiler-chosen inlining of the config-3 kernel: throughput at 65,536 documents for
# 6/7/8 waves per SIMD, and the instruction-cache counters of both builds. Every step is bounded.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-inl}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
D=${DOCS:-65536}
for NI in 1 0; do for W in ${WAVES:-7 6 8}; do
  MT_REPLAY_NOINLINE=$NI MT_REPLAY_WAVES=$W timeout -k 10 400 python -u bench.py --docs $D --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/ni${NI}_w$W.json" 2> "$OUT/ni${NI}_w$W.err" || { echo "ni $NI w $W rc=$?"; tail "$OUT/ni${NI}_w$W.err"; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/ni${NI}_w$W.json')); print('noinline $NI waves $W', round(d['value'] / 1e6, 2), 'Mops/s', round(d['roofline']['kernel_ms'], 1), 'ms')"
done; done
for NI in 1 0; do
  MT_REPLAY_NOINLINE=$NI timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY -d "$OUT/ic$NI" -o run --output-format csv -- python3 bench.py --docs 16384 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/ic$NI.json" 2> "$OUT/ic$NI.err" || { echo "icache pass $NI rc=$?"; exit 1; }
done
echo done
