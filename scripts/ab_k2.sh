#!/bin/bash
# K2 A/B on the GPU box: parity tests, then per-variant window timing under rocprofv3.
#   scripts/ab_k2.sh TAG "VAR1=.. VAR2=.." ...   (each quoted arg = one env variant)
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== variant $i: $v"
  ( [ -n "$v" ] && export $v; timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_${TAG}_$i -o run --output-format csv \
      -- python3 scripts/prof_window.py 6 > gpurun_out/ab_${TAG}_$i.log 2>&1 ) || { echo "rc=$?"; tail gpurun_out/ab_${TAG}_$i.log; exit 1; }
  grep "^window" gpurun_out/ab_${TAG}_$i.log | tail -2
  python3 scripts/kstats.py $(find gpurun_out/ab_${TAG}_$i -name '*kernel_stats.csv' | head -1) 8
done
