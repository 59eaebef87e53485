#!/bin/bash
# Full-size bench on one MI355X (bench.py defaults: config 3, 65,536 docs x 4,096 sequenced msgs),
# its rocprofv3 kernel-trace summary, and the HBM traffic counters (one PMC group per run).
TAG=${1:-bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
# a heartbeat under gpurun_out/ while long steps run (each step has its own time limit)
( while sleep 60; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
export TMPDIR=/tmp
ARGS=${ARGS:-}
timeout -k 10 600 python -u bench.py $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo "trace rc=$?"; tail -20 "$OUT/trace.err"; exit 1; }
cat "$OUT/trace.json"
if [ -n "$PMC" ]; then
  timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" || { echo "pmc fetch rc=$?"; exit 1; }
  timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err" || { echo "pmc write rc=$?"; exit 1; }
  echo pmc done
fi
