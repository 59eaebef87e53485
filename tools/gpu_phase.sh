#!/bin/bash
# GPU parity tests + per-phase cycle profile (tools/phase_profile.py); output under gpurun_out/.
TAG=${1:-x}
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.txt 2>&1 || { tail -30 gpurun_out/pt_$TAG.txt; exit 1; }
tail -2 gpurun_out/pt_$TAG.txt
timeout -k 10 300 python -u tools/phase_profile.py --docs ${DOCS:-2048} > gpurun_out/phase_$TAG.txt 2>&1 || { tail -30 gpurun_out/phase_$TAG.txt; exit 1; }
cat gpurun_out/phase_$TAG.txt
