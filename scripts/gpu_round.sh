#!/bin/bash
# GPU-box round check: parity tests, bench line, rocprofv3 kernel stats of the bench window.
#   scripts/gpu_round.sh TAG [skip-tests]
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/t_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/t_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 bench.py > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/b_$TAG.json
[ $rc -eq 0 ] || { tail -20 gpurun_out/b_$TAG.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python3 scripts/prof_window.py 6 > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "rocprof rc=$rc"
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" 16
exit $rc
