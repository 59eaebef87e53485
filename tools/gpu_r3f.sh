#!/bin/bash
# Round-3 check of the 126 KB replay kernel: GPU tests, the default config-3 bench with its kernel trace,
# FETCH_SIZE / WRITE_SIZE, SQ instruction / wait and instruction-cache passes, configs 2 and 5.
# Every GPU step is bounded; the chain stops at the first failure (the i-cache pass is optional).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r3f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
( while sleep 60; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|ERROR|Error" "$OUT/pytest_gpu.txt" | head -20; tail -5 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 600 python -u bench.py > "$OUT/c3.json" 2> "$OUT/c3.err" || { echo "bench rc=$?"; tail -20 "$OUT/c3.err"; exit 1; }
cat "$OUT/c3.json"
A="--steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo "trace rc=$?"; tail -20 "$OUT/trace.err"; exit 1; }
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py $A > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" || { echo "pmc fetch rc=$?"; exit 1; }
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py $A > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err" || { echo "pmc write rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d "$OUT/pmc_inst" -o run --output-format csv -- python3 bench.py $A > "$OUT/pmc_inst.json" 2> "$OUT/pmc_inst.err" || { echo "pmc inst rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d "$OUT/pmc_wait" -o run --output-format csv -- python3 bench.py $A > "$OUT/pmc_wait.json" 2> "$OUT/pmc_wait.err" || { echo "pmc wait rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d "$OUT/pmc_icache" -o run --output-format csv -- python3 bench.py --docs 16384 $A > "$OUT/pmc_icache.json" 2> "$OUT/pmc_icache.err" || echo "pmc icache rc=$? (optional)"
timeout -k 10 400 python -u bench.py --config 2 --steps 3 --warmup 1 > "$OUT/c2.json" 2> "$OUT/c2.err" || { echo "c2 rc=$?"; tail "$OUT/c2.err"; exit 1; }
timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err" || { echo "c5 rc=$?"; tail "$OUT/c5.err"; exit 1; }
for f in c2 c5; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f', round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],1), d['roofline']['frac'])"; done
