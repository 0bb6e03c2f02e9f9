#!/bin/bash
# last-block graphs: call-graph terms from every block's share (default) vs the last block's own
# chain (MR_TR_LFSSV=0) -- bitwise test, C3-sized one-window latency, C3 line
set -o pipefail
OUT=${OUT:-gpurun_out/lfssv}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rca.py -k "last_block or c3_window or layout_order or single_window" > $OUT/tests.txt 2>&1 || { tail -n 30 $OUT/tests.txt; exit 1; }
for v in 0 1 0 1; do
  MR_TR_LFSSV=$v timeout -k 10 180 python -u scripts/chunk_iso.py 40 1 500 20000 >> $OUT/c3w1_$v.txt 2>&1 || exit 1
done
for v in 0 1 0 1; do
  MR_TR_LFSSV=$v timeout -k 10 300 python3 bench.py --config c3 --no-traffic --no-cpu --no-side --steps 5 --warmup 1 >> $OUT/c3_$v.json 2>> $OUT/err.txt || exit 1
done
