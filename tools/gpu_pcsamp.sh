#!/bin/bash
# PC sampling (rocprofv3 beta) of the config-3 replay kernel on a small batch: which instructions
# the waves sit on. Lists the available PC-sampling configurations first; every step is bounded.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-pcs}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/list.txt" 2>&1; echo "list rc=$?"
grep -i -A6 "pc.sampl\|host_trap\|stochastic" "$OUT/list.txt" | head -40
M=${METHOD:-host_trap}
U=${UNIT:-time}
I=${INTERVAL:-1}
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U --pc-sampling-interval $I -d "$OUT/pc" -o run --output-format csv -- python3 bench.py --docs ${DOCS:-4096} --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pc.json" 2> "$OUT/pc.err"; rc=$?
echo "pc rc=$rc"; tail -5 "$OUT/pc.err"; ls -la "$OUT/pc" "$OUT"/pc/* 2>/dev/null | head -20
