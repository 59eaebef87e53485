#!/bin/bash
# One parametrised GPU runner (replaces the per-call tools/gpu_*.sh scripts).
#
#   tools/gpu.sh TAG STEP [STEP ...]
#
# Steps (run in order; every GPU step has its own time limit and the chain stops at the first failure):
#   tests[=EXPR]     pytest -m gpu (optionally -k EXPR)            -> OUT/pytest_gpu.txt
#   smoke            __graft_entry__ smoke()                        -> OUT/smoke.txt
#   bench:C          bench.py --config C (with CPU baseline)        -> OUT/bench_cC.json
#   trace:C          rocprofv3 --kernel-trace --stats of bench.py   -> OUT/trace_cC/ (+ kernel_stats.csv)
#   traffic:C        FETCH_SIZE pass + WRITE_SIZE pass              -> OUT/pmc_fetch_cC, OUT/pmc_write_cC
#   inst:C           SQ instruction-count pass                      -> OUT/pmc_inst_cC
#   wait:C           SQ wait / busy / LDS bank-conflict pass        -> OUT/pmc_wait_cC
#   icache:C         instruction-cache pass (SQC_ICACHE_*, SQ_IFETCH) -> OUT/pmc_icache_cC
#   phase:C          per-phase cycle clocks (profiling build)       -> OUT/phase_cC.txt
#   py:SCRIPT        python -u SCRIPT (a helper under tools/)       -> OUT/py_<name>.txt
#   ab:C:L1,L2,...   bench.py --config C per library build/Lk (MT_REPLAY_LIB), digests compared with L1
# Per-config extra bench arguments: ARGS_C (e.g. ARGS_4="--ops-per-doc 300000"); PHASE_C for phase:C.
# Generated workloads are cached under /tmp/mtgen between the steps of one call (bench.py --gen-cache).
set -o pipefail
export TMPDIR=/tmp
export MT_GEN_CACHE=${MT_GEN_CACHE:-/tmp/mtgen}
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
( while sleep 50; do date >> "$OUT/heartbeat"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT

fail() { echo "STEP $1 failed rc=$2"; [ -f "$3" ] && tail -25 "$3"; exit 1; }
bargs() { local v="ARGS_$1"; echo "--config $1 ${!v}"; }
prof_lim() { [ "$1" = 4 ] && echo 900 || echo 420; }

for S in "$@"; do
  K=${S%%[:=]*}
  A=${S#*[:=]}
  [ "$A" = "$S" ] && A=""
  echo "== $S ($(date +%T))"
  case $K in
    tests)
      SEL=()
      [ -n "$A" ] && SEL=(-k "$A")
      timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread "${SEL[@]}" \
        > "$OUT/pytest_gpu.txt" 2>&1 || fail "$S" $? "$OUT/pytest_gpu.txt"
      tail -1 "$OUT/pytest_gpu.txt" ;;
    smoke)
      timeout -k 10 300 python -u __graft_entry__.py smoke > "$OUT/smoke.txt" 2>&1 || fail "$S" $? "$OUT/smoke.txt"
      tail -1 "$OUT/smoke.txt" ;;
    bench)
      timeout -k 10 $(prof_lim "$A") python -u bench.py $(bargs "$A") > "$OUT/bench_c$A.json" 2> "$OUT/bench_c$A.err" \
        || fail "$S" $? "$OUT/bench_c$A.err"
      cat "$OUT/bench_c$A.json" ;;
    trace)
      timeout -k 10 $(prof_lim "$A") rocprofv3 --kernel-trace --stats -d "$OUT/trace_c$A" -o run --output-format csv \
        -- python3 bench.py $(bargs "$A") --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/trace_c$A.json" \
        2> "$OUT/trace_c$A.err" || fail "$S" $? "$OUT/trace_c$A.err"
      f=$(find "$OUT/trace_c$A" -name '*kernel_stats.csv' | head -1)
      cp "$f" "$OUT/trace_c${A}_kernel_stats.csv"; head -3 "$f" ;;
    traffic)
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL $(prof_lim "$A") rocprofv3 --pmc $C -d "$OUT/pmc_${C}_c$A" -o run --output-format csv \
          -- python3 bench.py $(bargs "$A") --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > "$OUT/pmc_${C}_c$A.json" \
          2> "$OUT/pmc_${C}_c$A.err" || fail "$S/$C" $? "$OUT/pmc_${C}_c$A.err"
      done ;;
    inst)
      timeout -s KILL $(prof_lim "$A") rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM \
        SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d "$OUT/pmc_inst_c$A" -o run --output-format csv \
        -- python3 bench.py $(bargs "$A") --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > "$OUT/pmc_inst_c$A.json" \
        2> "$OUT/pmc_inst_c$A.err" || fail "$S" $? "$OUT/pmc_inst_c$A.err" ;;
    wait)
      timeout -s KILL $(prof_lim "$A") rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d "$OUT/pmc_wait_c$A" -o run \
        --output-format csv -- python3 bench.py $(bargs "$A") --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
        > "$OUT/pmc_wait_c$A.json" 2> "$OUT/pmc_wait_c$A.err" || fail "$S" $? "$OUT/pmc_wait_c$A.err" ;;
    icache)
      timeout -s KILL $(prof_lim "$A") rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_IFETCH SQC_ICACHE_REQ \
        SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d "$OUT/pmc_icache_c$A" -o run \
        --output-format csv -- python3 bench.py $(bargs "$A") --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
        > "$OUT/pmc_icache_c$A.json" 2> "$OUT/pmc_icache_c$A.err" || fail "$S" $? "$OUT/pmc_icache_c$A.err" ;;
    phase)
      v="PHASE_$A"
      timeout -k 10 $(prof_lim "$A") python -u tools/phase_profile.py --config "$A" ${!v} > "$OUT/phase_c$A.txt" 2>&1 \
        || fail "$S" $? "$OUT/phase_c$A.txt"
      cat "$OUT/phase_c$A.txt" ;;
    ab)  # ab:C:libA,libB,... : one bench line per library (MT_REPLAY_LIB), digests compared with the first
      C=${A%%:*}; LIBS=${A#*:}
      first=""
      for L in ${LIBS//,/ }; do
        n=$(basename "$L" .so)
        MT_REPLAY_LIB=$PWD/fluidframework_amd/build/$L timeout -k 10 $(prof_lim "$C") python -u bench.py $(bargs "$C") \
          --no-cpu-baseline --no-e2e --digests-out "$OUT/dig_c${C}_$n.npy" > "$OUT/ab_c${C}_$n.json" 2> "$OUT/ab_c${C}_$n.err" \
          || fail "$S/$n" $? "$OUT/ab_c${C}_$n.err"
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,3), 'Mops/s', round(d['roofline']['kernel_ms'],1), 'ms')" "$OUT/ab_c${C}_$n.json" "$n"
        if [ -z "$first" ]; then first=$n; else
          python -c "import numpy as np,sys; a=np.load(sys.argv[1]); b=np.load(sys.argv[2]); print('  digests equal to', sys.argv[3], bool((a==b).all()))" "$OUT/dig_c${C}_$first.npy" "$OUT/dig_c${C}_$n.npy" "$first"
        fi
      done ;;
    py)
      n=$(basename "${A%% *}" .py)
      timeout -k 10 600 python -u $A > "$OUT/py_$n.txt" 2>&1 || fail "$S" $? "$OUT/py_$n.txt"
      tail -5 "$OUT/py_$n.txt" ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
