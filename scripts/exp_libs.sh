#!/bin/bash
# GPU box: C4 iteration time and k_fx_a phase stamps with alternative library builds (exp/).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in base ${LIBS:-e1 e2 e3}; do
  if [ $lib = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/exp/lib_$lib.so; fi
  MR_FX_STAMP=1 timeout -k 10 300 python3 bench.py --config c4 --c4-ops ${OPS:-10000} --steps 1 --warmup 1 > gpurun_out/x_$lib.json 2> gpurun_out/x_$lib.err || { tail -5 gpurun_out/x_$lib.err; exit 1; }
  echo "$lib $(grep stamp gpurun_out/x_$lib.err | tail -1 | cut -c1-220)"
done
