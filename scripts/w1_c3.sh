#!/bin/bash
# One C3-sized window per call (500 ops / 20k traces): host latency, default vs AB_ENV, interleaved,
# then a kernel trace of the default path's last call -> gpurun_out/w1c3_TAG*
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python3 scripts/chunk_iso.py 30 1 500 20000 2>/dev/null | sed "s/^/def$r /" || exit 1
  if [ -n "$AB_ENV" ]; then timeout -k 10 300 env $AB_ENV python3 scripts/chunk_iso.py 30 1 500 20000 2>/dev/null | sed "s/^/ab$r /" || exit 1; fi
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/w1c3_$TAG -o run --output-format csv -- python3 scripts/chunk_iso.py 10 1 500 20000 > /dev/null 2>&1 || exit 1
f=$(find gpurun_out/w1c3_$TAG -name '*kernel_trace.csv' | head -1)
python3 scripts/call_timeline.py "$f" > gpurun_out/w1c3_${TAG}_timeline.txt && tail -3 gpurun_out/w1c3_${TAG}_timeline.txt
rm -f "$f"
