#!/bin/bash
# A/B of alternative builds of the library (timing experiments): c4 (or $CFG) bench per build.
#   scripts/ab_lib.sh TAG dir1 dir2 ...   ("-" = the in-tree library)
TAG=$1; shift
CFG=${CFG:-c4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for d in "$@"; do
  if [ "$d" = "-" ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$GRAFT_REPO_ROOT/$d/libmicrorank_hip.so; fi
  n=$(echo "$d" | tr '/' '_')
  timeout -k 10 300 python3 bench.py --config $CFG --steps 5 --warmup 1 --no-traffic --no-cpu > gpurun_out/ab_${TAG}_$n.json 2> gpurun_out/ab_${TAG}_$n.err || { tail -5 gpurun_out/ab_${TAG}_$n.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['value'],d.get('windows_per_s'),r['avg_launch_us'],r['frac'])" gpurun_out/ab_${TAG}_$n.json "$d"
done
