set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "waves1 or waves-1 or occupancy" > gpurun_out/r06l/pytest.txt 2>&1 || { tail -30 gpurun_out/r06l/pytest.txt; exit 1; }
tail -1 gpurun_out/r06l/pytest.txt
for W in 4 1; do
  MT_SMALL_WAVES=$W timeout -k 10 300 python -u bench.py --config 1 --no-cpu-baseline --no-e2e --digests-out gpurun_out/r06l/dig_c1_w$W.npy > gpurun_out/r06l/c1_w$W.json 2> gpurun_out/r06l/c1_w$W.err || { tail -20 gpurun_out/r06l/c1_w$W.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,3), 'Mops/s', round(d['roofline']['kernel_ms'],2), 'ms')" gpurun_out/r06l/c1_w$W.json c1_w$W
done
python -c "import numpy as np; print('c1 digests equal', bool((np.load('gpurun_out/r06l/dig_c1_w4.npy')==np.load('gpurun_out/r06l/dig_c1_w1.npy')).all()))"
for D in 768 256; do for W in 4 1; do
  MT_SMALL_WAVES=$W timeout -k 10 300 python -u bench.py --config 3 --docs $D --no-cpu-baseline --no-e2e --digests-out gpurun_out/r06l/dig_c3_${D}_w$W.npy > gpurun_out/r06l/c3_${D}_w$W.json 2> gpurun_out/r06l/c3_${D}_w$W.err || { tail -20 gpurun_out/r06l/c3_${D}_w$W.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,3), 'Mops/s', round(d['roofline']['kernel_ms'],2), 'ms')" gpurun_out/r06l/c3_${D}_w$W.json c3_${D}_w$W
done; done
python -c "import numpy as np; print('c3 digests equal', bool((np.load('gpurun_out/r06l/dig_c3_768_w4.npy')==np.load('gpurun_out/r06l/dig_c3_768_w1.npy')).all()))"
