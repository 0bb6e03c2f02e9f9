#!/bin/bash
# GPU box: chosen test files (one process), log to gpurun_out/q_TAG.log
#   scripts/gpu_quick.sh TAG test_file...
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/q_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/q_$TAG.log | tail -40; exit $rc
