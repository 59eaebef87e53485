#!/bin/bash
# GPU tests, config 4 (one step, CPU-baseline sample), then the config-4 phase profile (256 docs x 300k).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-c4p}
OUT=gpurun_out/$TAG
bash tools/gpu_c4.sh "$TAG" || exit 1
timeout -k 10 400 python -u tools/phase_profile.py --config 4 --docs 256 --ops 300000 > "$OUT/phase_c4.txt" 2>&1 || { tail -20 "$OUT/phase_c4.txt"; exit 1; }
cat "$OUT/phase_c4.txt"
