#!/bin/bash
# GPU box: GPU tests, C4 bench, then rocprofv3 kernel stats of a short C4 run.
#   scripts/gpu_c4prof.sh TAG [skip-tests]
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 500 python3 bench.py --config c4 --steps 5 --warmup 1 --no-cpu > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err
rc=$?; echo "bench c4 rc=$rc"; cat gpurun_out/c4_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/c4_$TAG.err; exit $rc; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/c4p_$TAG -o run --output-format csv \
    -- python3 bench.py --config c4 --steps 4 --warmup 1 --no-cpu > gpurun_out/c4p_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find gpurun_out/c4p_$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" 14
exit $rc
