#!/bin/bash
# GPU box: C2 bench line at several concurrent-window stream counts.
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for w in ${WS:-1 2 4}; do
  timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --streams $w > gpurun_out/bs${w}_$TAG.json 2> gpurun_out/bs${w}_$TAG.err || { tail -5 gpurun_out/bs${w}_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bs${w}_$TAG.json'));print('W=$w', d['value'], 'GTEPS', d['windows_per_s'], 'win/s', d['ms_per_step'], 'ms/step', d['roofline']['avg_launch_us'], 'us/iter')"
done
