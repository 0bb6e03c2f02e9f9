#!/bin/bash
# GPU box: rocprof kernel stats of the C2 bench (default kernel vs MR_FX_V1), one stream
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in wv v1; do
  if [ $v = v1 ]; then export MR_FX_V1=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2p_${TAG}_$v -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-traffic --streams 1 > gpurun_out/c2p_${TAG}_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/c2p_${TAG}_$v.log; exit 1; }
  f=$(find gpurun_out/c2p_${TAG}_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"; python3 scripts/kstats.py "$f" 8
done
unset MR_FX_V1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4p_${TAG} -o run --output-format csv -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu --no-traffic > gpurun_out/c4p_${TAG}.log 2>&1 || { echo "c4 failed"; tail -3 gpurun_out/c4p_${TAG}.log; exit 1; }
f=$(find gpurun_out/c4p_${TAG} -name '*kernel_stats.csv' | head -1)
echo "== c4"; python3 scripts/kstats.py "$f" 8
