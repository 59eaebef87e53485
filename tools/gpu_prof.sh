#!/bin/bash
# Profiling pass on one MI355X: per-phase cycle profile (MT_PROF build), occupancy sweep of the
# config-3 kernel at the full 65,536 documents, the kernel-trace summary (CSV) and the PMC passes
# (instruction mix + waits, HBM fetch / write) of the default kernel. Every GPU step is bounded.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
D=${DOCS:-65536}
timeout -k 10 300 python -u tools/phase_profile.py --docs ${PDOCS:-8192} > "$OUT/phase.txt" 2>&1 || { echo "phase rc=$?"; tail -20 "$OUT/phase.txt"; exit 1; }
cat "$OUT/phase.txt"
for W in ${WAVES:-6 7 8}; do
  MT_REPLAY_WAVES=$W timeout -k 10 400 python -u bench.py --docs $D --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/occ_w$W.json" 2> "$OUT/occ_w$W.err" || { echo "occ $W rc=$?"; tail "$OUT/occ_w$W.err"; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/occ_w$W.json')); print('waves $W', round(d['value'] / 1e6, 2), 'Mops/s', round(d['roofline']['kernel_ms'], 1), 'ms')"
done
[ -n "$NOTRACE" ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --docs $D --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo "trace rc=$?"; tail -20 "$OUT/trace.err"; exit 1; }
find "$OUT/trace" -name '*kernel_stats.csv' -exec cat {} \;
[ -n "$NOPMC" ] && exit 0
P=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  P=$((P+1))
  timeout -s KILL 300 rocprofv3 --pmc $CTRS -d "$OUT/pmc$P" -o run --output-format csv -- python3 bench.py --docs ${PMCDOCS:-$D} --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc$P.json" 2> "$OUT/pmc$P.err" || { echo "pmc pass $P rc=$?"; exit 1; }
done
echo pmc done
