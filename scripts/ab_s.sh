#!/bin/bash
# GPU box: GPU tests, then C4 and C2 bench lines for each MR_FX_S value.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t_ab.log; [ $rc -eq 0 ] || exit $rc
fi
for sv in ${SV:-2 1}; do
  MR_FX_S=$sv timeout -k 10 300 python3 bench.py --config c4 --steps 2 --warmup 1 > gpurun_out/ab_c4_$sv.json 2> gpurun_out/ab_c4_$sv.err || { tail -5 gpurun_out/ab_c4_$sv.err; exit 1; }
  MR_FX_S=$sv timeout -k 10 300 python3 bench.py --no-traffic > gpurun_out/ab_c2_$sv.json 2> gpurun_out/ab_c2_$sv.err || { tail -5 gpurun_out/ab_c2_$sv.err; exit 1; }
  python3 -c "
import json
for c in ('c4','c2'):
    d=json.load(open('gpurun_out/ab_%s_$sv.json'%c)); print('S=$sv', c, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
