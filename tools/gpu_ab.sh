#!/bin/bash
# A/B of replay-kernel builds in one GPU call (MT_REPLAY_LIB=build/libmtreplay<suffix>.so), config 3 at
# DOCS documents; bounded, stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
( while sleep 60; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
A="--docs ${DOCS:-32768} --steps 3 --warmup 1 --no-cpu-baseline"
for T in ${VARIANTS:-base _v0}; do  # "base" = the in-tree libmtreplay.so
  V=$T; [ "$T" = base ] && V=""
  MT_REPLAY_LIB=$PWD/fluidframework_amd/build/libmtreplay$V.so timeout -k 10 300 python -u bench.py $A > "$OUT/c3$V.json" 2> "$OUT/c3$V.err" || { echo "bench $V rc=$?"; tail "$OUT/c3$V.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3$V.json'));print('lib$V', round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],1))"
done
