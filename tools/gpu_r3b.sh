#!/bin/bash
# Round-3 GPU check: GPU tests, then the default (config-3) bench with kernel trace, FETCH_SIZE /
# WRITE_SIZE passes and the SQ instruction / wait counters of the same kernel, then config 2 HBM- and
# LDS-resident. Every GPU step is bounded; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r3b}
TESTS_ONLY=1 bash tools/gpu_round.sh ${TAG}_tests || exit 1
PMC=1 bash tools/gpu_bench.sh ${TAG}_c3 || exit 1
python tools/merge_traffic.py gpurun_out/${TAG}_c3 > gpurun_out/${TAG}_c3/bench_traffic.json || exit 1
OUT=gpurun_out/${TAG}_c3
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d "$OUT/pmc_inst" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_inst.json" 2> "$OUT/pmc_inst.err" || { echo "pmc inst rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d "$OUT/pmc_wait" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_wait.json" 2> "$OUT/pmc_wait.err" || { echo "pmc wait rc=$?"; exit 1; }
timeout -k 10 400 python -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c2_hbm.json 2> gpurun_out/${TAG}_c2_hbm.err || { echo "c2 hbm rc=$?"; exit 1; }
MT_REPLAY_LDS=1 timeout -k 10 400 python -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c2_lds.json 2> gpurun_out/${TAG}_c2_lds.err || { echo "c2 lds rc=$?"; exit 1; }
cat gpurun_out/${TAG}_c2_hbm.json gpurun_out/${TAG}_c2_lds.json
