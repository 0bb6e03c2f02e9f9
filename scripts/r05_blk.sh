#!/bin/bash
# window-build block partition A/B: MR_LO_BLK_MIN (minimum blocks per table) on one-window
# latency (C2 / C3-sized) and on the C2 / C3 batch lines
set -o pipefail
OUT=${OUT:-gpurun_out/blk}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rca.py tests/test_gpu_graph_build.py > $OUT/tests.txt 2>&1 || { tail -n 30 $OUT/tests.txt; exit 1; }
for v in 0 256 1024 0 256 1024; do
  MR_LO_BLK_MIN=$v timeout -k 10 180 python -u scripts/chunk_iso.py 30 1 >> $OUT/c2w1_$v.txt 2>&1 || exit 1
  MR_LO_BLK_MIN=$v timeout -k 10 180 python -u scripts/chunk_iso.py 30 1 500 20000 >> $OUT/c3w1_$v.txt 2>&1 || exit 1
done
for v in 0 256 1024; do
  MR_LO_BLK_MIN=$v timeout -k 10 300 python3 bench.py --config c3 --no-traffic --no-cpu --no-side --steps 5 --warmup 1 >> $OUT/c3_$v.json 2>> $OUT/err.txt || exit 1
  MR_LO_BLK_MIN=$v timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --no-c4-leg --no-side --steps 5 --warmup 1 >> $OUT/c2_$v.json 2>> $OUT/err.txt || exit 1
done
