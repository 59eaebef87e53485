#!/bin/bash
# GPU tests (parallel getText), then the default line with its HBM traffic counters (tools/gpu_bench.sh PMC=1).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2m}
TESTS_ONLY=1 bash tools/gpu_round.sh $TAG || exit 1
PMC=1 bash tools/gpu_bench.sh $TAG/pmc || exit 1
python3 tools/merge_traffic.py gpurun_out/$TAG/pmc | tail -3
