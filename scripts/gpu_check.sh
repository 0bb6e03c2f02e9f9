#!/bin/bash
# GPU-box check: parity tests, then a K2 timing run.  Usage: scripts/gpu_check.sh TAG [pytest-args]
TAG=${1:-x}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q "$@" > gpurun_out/t_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || exit $rc
ROLE_AB=1 timeout -k 10 300 python3 scripts/prof_pagerank.py 1000 200000 10 > gpurun_out/p_$TAG.log 2>&1
rc=$?
grep -v "^W20\|^E20" gpurun_out/p_$TAG.log
exit $rc
