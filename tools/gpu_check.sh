#!/bin/bash
# One GPU-box pass: GPU parity tests, smoke, a short bench and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-check}
shift || true
DOCS=${DOCS:-4096}
mkdir -p "$OUT"
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { echo "smoke failed rc=$?"; tail -30 "$OUT/smoke.txt"; exit 1; }
timeout -k 10 300 python -u bench.py --docs $DOCS --steps 3 --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --docs $DOCS --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { echo "rocprof failed rc=$?"; tail -30 "$OUT/prof_bench.err"; exit 1; }
tail -3 "$OUT/pytest_gpu.txt"; cat "$OUT/smoke.txt" | tail -2; cat "$OUT/bench.json"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \;
# optional PMC passes (one counter group per run; each bounded)
if [ -n "$PMC" ]; then
  P=0
  for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
              "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT" \
              "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    P=$((P+1))
    timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$OUT/pmc$P" -o run --output-format csv -- python3 bench.py --docs $DOCS --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc${P}.json" 2> "$OUT/pmc${P}.err" || { echo "pmc pass $P failed rc=$?"; exit 1; }
  done
  echo "pmc done"
fi
