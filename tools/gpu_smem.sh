#!/bin/bash
# Round-2 SMEM root-cause run: the addressing-form probe, then the round-1 failing case with the
# compiler barrier removed (libmtreplay_noclob.so), each step bounded; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-smem}
mkdir -p "$OUT"
timeout -k 10 120 ./fluidframework_amd/build/smem_probe 262144 > "$OUT/probe.txt" 2>&1; echo "probe rc=$?" >> "$OUT/probe.txt"
cat "$OUT/probe.txt"
MT_REPLAY_LIB=fluidframework_amd/build/libmtreplay_noclob.so timeout -k 10 300 python -u tools/gpu_baddocs.py config2 2000 96 > "$OUT/noclob_baddocs.txt" 2>&1 || { echo "baddocs rc=$?"; tail -20 "$OUT/noclob_baddocs.txt"; exit 1; }
cat "$OUT/noclob_baddocs.txt"
