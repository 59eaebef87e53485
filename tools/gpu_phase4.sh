#!/bin/bash
# Per-phase cycle profile (profiling build, -DMT_PROF) of the config-4 tiled kernel; output under gpurun_out/.
TAG=${1:-c4}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/phase_profile.py --config 4 --docs ${DOCS:-256} --ops ${OPS:-300000} > gpurun_out/phase_$TAG.txt 2>&1 || { tail -30 gpurun_out/phase_$TAG.txt; exit 1; }
cat gpurun_out/phase_$TAG.txt
