#!/bin/bash
# GPU box: C2 window bench with k_fx_a phase stamps at the given TT caps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for tt in ${TTS:-1024 512}; do
  MR_TT=$tt MR_FX_STAMP=1 timeout -k 10 300 python3 bench.py --no-traffic --steps 2 --warmup 1 > gpurun_out/c2s_$tt.json 2> gpurun_out/c2s_$tt.err || { tail -5 gpurun_out/c2s_$tt.err; exit 1; }
  echo "TT=$tt"; grep stamp gpurun_out/c2s_$tt.err | tail -2
done
