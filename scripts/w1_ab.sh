#!/bin/bash
# GPU box: one-window latency (bench.py window_ms, W = 1) of C3 and C2 for the default library and
# the A/B libraries (VARIANTS="def ab ab2": libmicrorank_hip_<v>.so)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-def ab}; do
  if [ $v != def ]; then export MR_LIB_PATH=$PWD/microrank_amd/libmicrorank_hip_$v.so; else unset MR_LIB_PATH; fi
  for c in c3 c2; do
    timeout -k 10 300 python3 bench.py --config $c --no-traffic --no-cpu --no-c4-leg --steps 1 --warmup 1 --c2-distinct 8 > gpurun_out/w1ab_${v}_$c.json 2> gpurun_out/w1ab_${v}_$c.err || { tail -5 gpurun_out/w1ab_${v}_$c.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], d.get('window_ms'))" gpurun_out/w1ab_${v}_$c.json $v $c
  done
done
unset MR_LIB_PATH
