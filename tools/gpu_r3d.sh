#!/bin/bash
# Round-3 occupancy re-sweep of the config-3 kernel after the spill work (16,384 docs: two resident
# rounds of 8,192 waves), and memory-pipeline counters of the default build. Bounded, stops at a failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3d
mkdir -p "$OUT"
( while sleep 60; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { echo "smoke rc=$?"; tail "$OUT/smoke.txt"; exit 1; }
A="--docs 16384 --steps 2 --warmup 1 --no-cpu-baseline"
for V in "" _w7 _w6; do
  MT_REPLAY_LIB=$PWD/fluidframework_amd/build/libmtreplay$V.so timeout -k 10 300 python -u bench.py $A > "$OUT/c3$V.json" 2> "$OUT/c3$V.err" || { echo "bench $V rc=$?"; tail "$OUT/c3$V.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3$V.json'));print('$V', round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],1))"
done
timeout -s KILL 240 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/pmc_ta" -o run --output-format csv -- python3 bench.py $A > "$OUT/pmc_ta.json" 2> "$OUT/pmc_ta.err" || { echo "pmc ta rc=$?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc_tcc" -o run --output-format csv -- python3 bench.py $A > "$OUT/pmc_tcc.json" 2> "$OUT/pmc_tcc.err" || { echo "pmc tcc rc=$?"; exit 1; }
echo done
