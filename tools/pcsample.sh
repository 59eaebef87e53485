#!/bin/bash
# PC sampling of the replay kernel (rocprofv3, host-trap method): where the waves' instructions are, dynamically.
#   tools/pcsample.sh TAG CONFIG [bench args]  -> gpurun_out/TAG/pcs_cC/ (+ avail.txt: the box's PC-sampling configs)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:?tag}; C=${2:?config}; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || echo "list rc=$?"
timeout -k 10 600 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval ${PCS_INTERVAL:-50} -d "$OUT/pcs_c$C" -o run --output-format csv \
  -- python3 bench.py --config "$C" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e "$@" > "$OUT/pcs_c$C.json" \
  2> "$OUT/pcs_c$C.err" || { echo "pc sampling rc=$?"; tail -20 "$OUT/pcs_c$C.err"; exit 1; }
find "$OUT/pcs_c$C" -type f | head
