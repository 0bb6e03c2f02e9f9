#!/bin/bash
# GPU box: kernel stats of isolated window-batch calls (scripts/prof_batch.py W R) -> gpurun_out/pw_TAG
TAG=$1; W=${2:-8}; R=${3:-20}; OPS=${4:-500}; TR=${5:-20000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MR_WIN_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pw_$TAG -o run --output-format csv \
    -- python3 scripts/prof_batch.py $W $R $OPS $TR > gpurun_out/pw_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/pw_$TAG.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pw_$TAG -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py "$f" 30
find gpurun_out/pw_$TAG -name '*kernel_trace.csv' -delete
