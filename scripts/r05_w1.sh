#!/bin/bash
# single-window latency A/B: spectrum queued early vs after the PageRank words (C2 / C3-sized)
set -o pipefail
OUT=${OUT:-gpurun_out/w1}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rca.py -k "single_window_early or rerun_sets_up" > $OUT/tests.txt 2>&1 &&
for v in 0 1 0 1; do
  MR_WIN_SPEC_EARLY=$v timeout -k 10 180 python -u scripts/chunk_iso.py 40 1 >> $OUT/c2_spec$v.txt 2>&1 || exit 1
  MR_WIN_SPEC_EARLY=$v timeout -k 10 180 python -u scripts/chunk_iso.py 40 1 500 20000 >> $OUT/c3_spec$v.txt 2>&1 || exit 1
done
MR_WIN_PHASES=1 timeout -k 10 180 python -u scripts/chunk_iso.py 20 1 > $OUT/c2_phases.txt 2>&1
