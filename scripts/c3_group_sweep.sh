#!/bin/bash
# GPU box: C3 batch line at several window-group sizes (MR_WIN_GROUP; 0: the default rule)
#   scripts/c3_group_sweep.sh "0 256 512"
LIST=${1:-"0 256 512"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for g in $LIST; do
  E=""; [ "$g" != 0 ] && E="MR_WIN_GROUP=$g"
  timeout -k 10 300 env $E python3 bench.py --config c3 --no-traffic --no-cpu --no-side --steps 3 --warmup 1 > gpurun_out/c3g_$g.json 2> gpurun_out/c3g_$g.err || { tail -5 gpurun_out/c3g_$g.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print('group', sys.argv[2], d['value'], d.get('windows_per_s'), r.get('avg_launch_us'), r.get('frac'), r.get('bytes_per_launch'))" gpurun_out/c3g_$g.json $g
done
