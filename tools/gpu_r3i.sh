#!/bin/bash
# Per-phase cycle profile of the config-3 kernel at full occupancy (profiling build: -DMT_PROF) and the
# SQ instruction / wait counters of the adopted build. Bounded; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3i
mkdir -p "$OUT"
( while sleep 60; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u tools/phase_profile.py --docs ${DOCS:-65536} > "$OUT/phase.txt" 2>&1 || { tail -30 "$OUT/phase.txt"; exit 1; }
cat "$OUT/phase.txt"
A="--steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d "$OUT/pmc_inst" -o run --output-format csv -- python3 bench.py $A > "$OUT/pmc_inst.json" 2> "$OUT/pmc_inst.err" || { echo "pmc inst rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d "$OUT/pmc_wait" -o run --output-format csv -- python3 bench.py $A > "$OUT/pmc_wait.json" 2> "$OUT/pmc_wait.err" || { echo "pmc wait rc=$?"; exit 1; }
echo done
