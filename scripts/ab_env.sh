#!/bin/bash
# GPU box: C2 / C3 bench lines under values of one environment knob
#   VAR=MR_IX_BLOCKS VALS="64 128 256" scripts/ab_env.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in $VALS; do
  for cfg in ${CFGS:-c2 c3}; do
    env "$VAR=$v" timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-traffic > gpurun_out/ab_${cfg}_$v.json 2> gpurun_out/ab_${cfg}_$v.err || { echo "$v $cfg failed"; tail -3 gpurun_out/ab_${cfg}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['value'], d.get('windows_per_s'), r['avg_launch_us'], r['frac'])" gpurun_out/ab_${cfg}_$v.json $v $cfg
  done
done
