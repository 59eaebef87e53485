set -o pipefail
export TMPDIR=/tmp MT_GEN_CACHE=/tmp/mtgen
O=gpurun_out/r05b; mkdir -p $O
( while sleep 50; do date >> $O/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
for a in "3 cost 65536" "3 doc 65536" "3 cost 8192" "3 doc 8192" "2 cost 4096" "2 doc 4096"; do set -- $a
  timeout -k 10 400 python -u bench.py --config $1 --order $2 --docs $3 --no-cpu-baseline > $O/b_c$1_$2_$3.json 2> $O/b_c$1_$2_$3.err || { tail -20 $O/b_c$1_$2_$3.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,2), 'Mops/s', round(d['roofline']['kernel_ms'],1), 'ms', d['doc_time_ms'])" $O/b_c$1_$2_$3.json
done
