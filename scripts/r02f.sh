#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r02f.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_r02f.log; [ $rc -eq 0 ] || exit $rc
bash scripts/exp_c4.sh r02f
