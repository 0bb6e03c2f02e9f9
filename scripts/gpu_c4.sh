#!/bin/bash
# GPU box: full GPU tests, the default C2 bench line, and the C4 sharded bench at 1 GPU.
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err
rc=$?; echo "bench c2 rc=$rc"; cat gpurun_out/b_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/b_$TAG.err; exit $rc; }
timeout -k 10 500 python3 bench.py --config c4 --steps 5 --warmup 1 > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err
rc=$?; echo "bench c4 rc=$rc"; cat gpurun_out/c4_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/c4_$TAG.err; exit $rc; }
