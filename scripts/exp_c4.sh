#!/bin/bash
# GPU box: C4 bench against experiment builds of the library (xlib/libmr_exp*.so, MR_EXP bits:
# 1 no atomics, 2 no su gathers, 4 no X reads)
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in default xlib/libmr_exp*.so; do
  if [ $lib != default ]; then export MR_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-traffic > gpurun_out/x_$TAG.json 2> gpurun_out/x_$TAG.err || { echo "$lib failed"; tail -3 gpurun_out/x_$TAG.err; exit 1; }
  echo "$lib: $(python3 -c "import json;d=json.load(open('gpurun_out/x_$TAG.json'));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'])")"
done
