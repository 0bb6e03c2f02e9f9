#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for m in 1 0; do
  for cfg in c2 c3; do
    MR_PR_PERSIST=$m timeout -k 10 300 python3 bench.py --config $cfg --no-traffic --no-cpu --steps 5 --warmup 2 > gpurun_out/ab_${cfg}_p$m.json 2> gpurun_out/ab_${cfg}_p$m.err || { tail -5 gpurun_out/ab_${cfg}_p$m.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${cfg}_p$m.json'));r=d['roofline'];print('$cfg p$m', d['value'], d['windows_per_s'], r['avg_launch_us'], r['frac'], d['window_ms']['median'])"
  done
done
