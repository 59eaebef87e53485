#!/bin/bash
# Replay throughput of the small profile, HBM-resident, at 6 / 8 / 7 (default) waves per SIMD.
export TMPDIR=/tmp
D=${DOCS:-16384}
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --docs $D --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/occ_$name.json 2> gpurun_out/occ_$name.err || { tail gpurun_out/occ_$name.err; exit 1; }
  python3 -c "import json; d = json.load(open('gpurun_out/occ_$name.json')); print('$name', round(d['value'] / 1e6, 2), 'Mops/s', round(d['ms_per_step'], 1), 'ms')"
}
run hbm6 MT_REPLAY_WAVES=6
run hbm8 MT_REPLAY_WAVES=8
run hbm7 MT_REPLAY_WAVES=7
