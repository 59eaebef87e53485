set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "submit or napi or arena_gc" > gpurun_out/r06d/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r06d/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/r06d/pytest_gpu.txt
timeout -k 10 300 node tools/facade_latency.js 65536 200 > gpurun_out/r06d/facade_latency_65536.json 2> gpurun_out/r06d/facade_latency.err || { tail gpurun_out/r06d/facade_latency.err; exit 1; }
cat gpurun_out/r06d/facade_latency_65536.json
