#!/bin/bash
# GPU box: full GPU tests, C4 and C5 (12.5M traces) bench lines.
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/t_$TAG.log | tail -8; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py --config c4 --steps 5 --warmup 1 --no-cpu > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err
rc=$?; echo "bench c4 rc=$rc"; cut -c1-300 gpurun_out/c4_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/c4_$TAG.err; exit $rc; }
SMALL=12500000 NOFULL=1 bash scripts/gpu_c5.sh $TAG skip-tests
