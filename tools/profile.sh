#!/bin/bash
# Profiles bench.py on one GPU: kernel trace + stats, then PMC passes (one per counter group).
# Usage (on the GPU box, from the repo root): tools/profile.sh OUTDIR [bench args...]
set -u
OUT=${1:-gpurun_out/prof}
shift || true
ARGS=${@:---docs 4096 --steps 2 --warmup 1 --no-cpu-baseline}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit 11
P=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT" \
            "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  P=$((P+1))
  timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$OUT/pmc$P" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc${P}_bench.json" 2> "$OUT/pmc${P}_bench.err" || echo "pmc pass $P failed rc=$?"
done
exit 0
