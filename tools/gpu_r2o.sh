#!/bin/bash
# GPU tests (node: references / reconnect through the facade), then the occupancy re-sweep.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r2o}
TESTS_ONLY=1 bash tools/gpu_round.sh $TAG || exit 1
bash tools/gpu_r2n.sh $TAG/sweep || exit 1
