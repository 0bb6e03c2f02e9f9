#!/bin/bash
# GPU box: kernel trace of a bench run -> busy union / concurrency / kernel shares of its last SPAN ms
#   scripts/gpu_busy.sh TAG SPAN_MS [bench args...]
TAG=$1; SPAN=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/kb_$TAG -o run --output-format csv \
    -- python3 bench.py --no-traffic "$@" > gpurun_out/kb_$TAG.json 2> gpurun_out/kb_$TAG.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/kb_$TAG -name '*kernel_trace.csv' | head -1)
python3 scripts/ktrace_busy.py "$f" $SPAN 22 | tee gpurun_out/kb_$TAG.txt
rm -f "$f"
