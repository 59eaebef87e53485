#!/bin/bash
# Round-3 HEAD baseline: GPU tests, then the default bench with kernel trace and FETCH/WRITE passes.
set -o pipefail
export TMPDIR=/tmp
TESTS_ONLY=1 bash tools/gpu_round.sh r3a_head || exit 1
PMC=1 bash tools/gpu_bench.sh r3a_head_c3 || exit 1
python tools/merge_traffic.py gpurun_out/r3a_head_c3
