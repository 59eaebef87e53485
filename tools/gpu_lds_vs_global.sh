#!/bin/bash
# Same bench with the small-profile hot image in LDS (default) and in HBM (MT_REPLAY_GLOBAL=1).
export TMPDIR=/tmp
D=${DOCS:-16384}
timeout -k 10 400 python -u bench.py --docs $D --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/lvg_lds.json 2> gpurun_out/lvg_lds.err || { tail gpurun_out/lvg_lds.err; exit 1; }
MT_REPLAY_GLOBAL=1 timeout -k 10 400 python -u bench.py --docs $D --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/lvg_glb.json 2> gpurun_out/lvg_glb.err || { tail gpurun_out/lvg_glb.err; exit 1; }
python3 -c "
import json
for f in ('lds', 'glb'):
    d = json.load(open('gpurun_out/lvg_%s.json' % f)); print(f, round(d['value'] / 1e6, 2), 'Mops/s', round(d['ms_per_step'], 1), 'ms')
"
