#!/bin/bash
# A/B of environment settings on a window config: throughput and single-window latency per setting
#   CFG=c3 scripts/ab_lat.sh TAG "" "MR_X=1" ...
TAG=$1; shift
CFG=${CFG:-c3}; EXTRA=${EXTRA:-"--steps 5 --warmup 1"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python3 bench.py --config $CFG $EXTRA --no-traffic --no-cpu > gpurun_out/abl_${TAG}_$i.json 2> gpurun_out/abl_${TAG}_$i.err || { tail -5 gpurun_out/abl_${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(repr(sys.argv[2]),d['value'],d.get('windows_per_s'),r['avg_launch_us'],r['frac'],d.get('window_ms'))" gpurun_out/abl_${TAG}_$i.json "$e"
done
