#!/bin/bash
# GPU box: GPU tests, then the C5 bench (tile-path sharded iteration) at the 8-GPU per-rank share
# and at the full 100M traces on one GPU.   scripts/gpu_c5.sh TAG [skip-tests]
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python3 -u bench.py --config c5 --c4-traces ${SMALL:-12500000} --steps 3 --warmup 1 > gpurun_out/c5s_$TAG.json 2> gpurun_out/c5s_$TAG.err
rc=$?; echo "bench c5 small rc=$rc"; cat gpurun_out/c5s_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/c5s_$TAG.err; exit $rc; }
[ -n "$NOFULL" ] && exit 0
timeout -k 10 700 python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err
rc=$?; echo "bench c5 rc=$rc"; cat gpurun_out/c5_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/c5_$TAG.err; exit $rc; }
