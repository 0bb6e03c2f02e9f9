#!/bin/bash
# GPU box: selected GPU test files (args), then the W=1 window latency script
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/quick.log 2>&1 || { tail -30 gpurun_out/quick.log; exit 1; }
tail -2 gpurun_out/quick.log
bash scripts/w1.sh
