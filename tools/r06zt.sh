#!/bin/bash
# round-6 A/B of the ramped first chunks of mt_engine_submit_run (MT_SUBMIT_RAMP=1, default) against equal chunks (0):
# config-3 end-to-end rate, digests checked inside bench.py against the kernel-only replay
set -o pipefail
export TMPDIR=/tmp MT_GEN_CACHE=/tmp/mtgen
OUT=gpurun_out/r06zt
mkdir -p $OUT
for t in 0 1 0 1; do
  MT_SUBMIT_RAMP=$t timeout -k 10 420 python -u bench.py --config 3 --no-cpu-baseline > $OUT/e2e_ramp$t.json 2> $OUT/e2e_ramp$t.err \
    || { tail -20 $OUT/e2e_ramp$t.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['end_to_end']; print('ramp', sys.argv[2], round(d['value']/1e6,1), 'kernel', {k: (round(v['value']/1e6,1), v['digests_equal']) for k, v in e['modes'].items()})" $OUT/e2e_ramp$t.json $t
  cp $OUT/e2e_ramp$t.json $OUT/e2e_ramp${t}_$(date +%s).json
done
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -k "submit" > $OUT/pytest_submit.txt 2>&1 || { tail -20 $OUT/pytest_submit.txt; exit 1; }
tail -1 $OUT/pytest_submit.txt
