#!/bin/bash
# f3 streaming append: parity tests, then the stream bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rca.py -k "stream or append" > gpurun_out/stream_tests.log 2>&1 || { tail -40 gpurun_out/stream_tests.log; exit 1; }
tail -3 gpurun_out/stream_tests.log
timeout -k 10 600 python -u bench.py --config stream > gpurun_out/stream_bench.json 2> gpurun_out/stream_bench.err || { tail -30 gpurun_out/stream_bench.err; exit 1; }
cat gpurun_out/stream_bench.json
