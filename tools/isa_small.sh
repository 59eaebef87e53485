#!/bin/bash
# Analysis build of one config-3 replay kernel variant alone (VARIANT=w8|lds|dl): resource usage (register and
# spill counts) and the gfx950 assembly, in a minute instead of the full library's several.
# usage: tools/isa_small.sh OUTDIR [extra hipcc flags]
set -e
SRC=$(cd "$(dirname "$0")/.." && pwd)/fluidframework_amd/csrc/mt_small_${VARIANT:-w8}.hip
OUT=${1:-/tmp/isa}; shift || true
mkdir -p "$OUT"
cd "$OUT"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c --offload-device-only "$@" \
  -Rpass-analysis=kernel-resource-usage --save-temps "$SRC" \
  -o small.o > resource.txt 2>&1
grep -A12 "Function Name: _Z8k_replay" resource.txt | grep -E "SGPRs|VGPRs|Scratch|Occupancy|Spill" || true
