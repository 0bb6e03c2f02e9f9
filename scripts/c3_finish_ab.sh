#!/bin/bash
# GPU box: C3 batch line with the default finish, MR_TR_PF=0 and MR_TR_LASTFIN=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in def pf0 lf0; do
  E=""; [ $v = pf0 ] && E="MR_TR_PF=0"; [ $v = lf0 ] && E="MR_TR_LASTFIN=0"
  timeout -k 10 300 env $E python3 bench.py --config c3 --no-traffic --no-cpu --no-side --steps 3 --warmup 1 > gpurun_out/c3ab_$v.json 2> gpurun_out/c3ab_$v.err || { tail -5 gpurun_out/c3ab_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2], d['value'], d.get('windows_per_s'), r.get('avg_launch_us'), r.get('frac'))" gpurun_out/c3ab_$v.json $v
done
