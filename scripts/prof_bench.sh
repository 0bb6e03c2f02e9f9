#!/bin/bash
# GPU box: rocprofv3 kernel stats of a bench command -> gpurun_out/pb_TAG/ + top kernels
#   scripts/prof_bench.sh TAG [bench args...]
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pb_$TAG -o run --output-format csv \
    -- python3 bench.py --no-traffic "$@" > gpurun_out/pb_$TAG.json 2> gpurun_out/pb_$TAG.err
rc=$?
echo "rocprof rc=$rc"; cat gpurun_out/pb_$TAG.json
f=$(find gpurun_out/pb_$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" 30
exit $rc
