#!/bin/bash
# The whole round-end check in one call: GPU tests, config 3 (+ kernel trace), 2, 5, 4 (tools/gpu_r3h.sh),
# then the config-4 phase profile (256 docs x 300k). Bounded; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-full}
OUT=gpurun_out/$TAG
bash tools/gpu_r3h.sh "$TAG" || exit 1
timeout -k 10 400 python -u tools/phase_profile.py --config 4 --docs 256 --ops 300000 > "$OUT/phase_c4.txt" 2>&1 || { tail -20 "$OUT/phase_c4.txt"; exit 1; }
cat "$OUT/phase_c4.txt"
