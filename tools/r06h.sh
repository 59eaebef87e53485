#!/bin/bash
# round-6 A/B of the two-wave config-4 window pass (MT_WIN_HELPER) + the wave synchronization probe + the GPU suite
set -o pipefail
OUT=gpurun_out/r06h
mkdir -p $OUT
timeout -k 5 60 tools/bin/wave_sync_probe > $OUT/wave_sync.json || exit 1
cat $OUT/wave_sync.json
MT_REPLAY_LIB=$PWD/fluidframework_amd/build/libmt_wh2.so timeout -k 10 600 python -u -m pytest tests -x -v -m gpu \
  --timeout 300 --timeout-method thread -k "c4_large or tiled" > $OUT/pytest_wh.txt 2>&1 || { tail -30 $OUT/pytest_wh.txt; exit 1; }
tail -1 $OUT/pytest_wh.txt
ARGS_4="--ops-per-doc 300000" tools/gpu.sh r06h ab:4:libmtreplay.so,libmt_wh2.so
