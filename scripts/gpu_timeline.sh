#!/bin/bash
# GPU box: kernel trace of a bench run -> a bucketed timeline of SPAN ms from the timed steps
#   scripts/gpu_timeline.sh TAG SPAN_MS BUCKET_US [bench args...]
TAG=$1; SPAN=$2; BK=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/kt_$TAG -o run --output-format csv \
    -- python3 bench.py --no-traffic "$@" > gpurun_out/kt_$TAG.json 2> gpurun_out/kt_$TAG.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/kt_$TAG -name '*kernel_trace.csv' | head -1)
head -1 "$f"
python3 scripts/ktrace_busy.py "$f" 0 8
python3 scripts/ktrace_timeline.py "$f" $SPAN $BK > gpurun_out/kt_$TAG.txt
rm -f "$f"
