#!/bin/bash
# GPU box: rocprofv3 HIP API trace stats of a bench command -> gpurun_out/pa_TAG/ + top API calls
#   scripts/prof_api.sh TAG [bench args...]
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --hip-trace --stats -d gpurun_out/pa_$TAG -o run --output-format csv \
    -- python3 bench.py --no-traffic --no-cpu "$@" > gpurun_out/pa_$TAG.json 2> gpurun_out/pa_$TAG.err
rc=$?
echo "rocprof rc=$rc"
f=$(find gpurun_out/pa_$TAG -name '*hip_api_stats.csv' | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" 25
exit $rc
