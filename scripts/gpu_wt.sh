#!/bin/bash
# GPU box: quick C2 window A/B: bench line (no PMC, no CPU) + MR_WIN_TIMING phases.
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $TESTS > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 bench.py --no-traffic --no-cpu > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { tail -5 gpurun_out/b_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b_$TAG.json'));print('C2', d['value'], 'GTEPS', d['ms_per_step'], 'ms/window', d['roofline']['avg_launch_us'], 'us/iter')"
MR_WIN_TIMING=1 timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --steps 3 --warmup 1 > /dev/null 2> gpurun_out/wt_$TAG.err || exit 1
grep -v "^\[window\] detect [0-9.]* build_n [0-9]\{4\}" gpurun_out/wt_$TAG.err | tail -8
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
      -- python3 scripts/prof_window.py 6 > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
  f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1); python3 scripts/kstats.py "$f" 20
fi
if [ -n "$HIPTRACE" ]; then
  timeout -k 10 300 rocprofv3 --hip-trace --stats -d gpurun_out/hip_$TAG -o run --output-format csv \
      -- python3 scripts/prof_window.py 6 > gpurun_out/hip_$TAG.log 2>&1 || { tail -5 gpurun_out/hip_$TAG.log; exit 1; }
  f=$(find gpurun_out/hip_$TAG -name '*hip_api_stats.csv' | head -1); echo "== $f"; head -25 "$f" | cut -d, -f1-8
fi
