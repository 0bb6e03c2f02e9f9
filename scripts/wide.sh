#!/bin/bash
# wide fused path: parity tests, then the C5 bench line and its kernel table
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_pagerank.py tests/test_gpu_shard.py -k "wide or large_op" \
  > gpurun_out/wide_tests.log 2>&1 || { tail -40 gpurun_out/wide_tests.log; exit 1; }
tail -5 gpurun_out/wide_tests.log
if [ "$1" = "bench" ]; then
  timeout -k 10 700 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu > gpurun_out/c5_wide.json 2> gpurun_out/c5_wide.err || { tail -20 gpurun_out/c5_wide.err; exit 1; }
  cat gpurun_out/c5_wide.json
fi
