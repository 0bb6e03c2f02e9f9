#!/bin/bash
# one-window path: window tests, a C3-sized kernel trace, one-window latency (C3-sized / C2 / C3-sized)
set -o pipefail
OUT=${OUT:-gpurun_out/w1c3b}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rca.py > $OUT/tests.txt 2>&1 || { tail -n 20 $OUT/tests.txt; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 scripts/chunk_iso.py 10 1 500 20000 > $OUT/out.txt 2>&1 || exit 1
timeout -k 10 120 python3 scripts/chunk_iso.py 40 1 500 20000 >> $OUT/out.txt 2>&1 &&
timeout -k 10 120 python3 scripts/chunk_iso.py 40 1 >> $OUT/out.txt 2>&1 &&
timeout -k 10 120 python3 scripts/chunk_iso.py 40 1 500 20000 >> $OUT/out.txt 2>&1
