#!/bin/bash
# Memory-pipeline counters of the config-3 kernel (L1 TLB, L1->L2 latency, TA busy, L2 hits,
# vector-memory latency), one counter group per bounded run.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-mem}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
D=${DOCS:-65536}
P=0
for CTRS in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
            "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"; do
  P=$((P+1))
  timeout -s KILL 300 rocprofv3 --pmc $CTRS -d "$OUT/pmc$P" -o run --output-format csv -- python3 bench.py --docs $D --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc$P.json" 2> "$OUT/pmc$P.err" || { echo "pmc pass $P rc=$?"; tail -5 "$OUT/pmc$P.err"; exit 1; }
  echo "pass $P ok"
done
