#!/bin/bash
# GPU box: one bench config under several values of one environment knob
#   VALS="4 8 16" scripts/sweep_env.sh VAR [bench args...]
VAR=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python3 bench.py --no-cpu --no-traffic "$@" > gpurun_out/sw_$v.json 2> gpurun_out/sw_$v.err || { echo "$v failed"; tail -3 gpurun_out/sw_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d.get('windows_per_s'), d['roofline']['avg_launch_us'])" gpurun_out/sw_$v.json $VAR $v
done
