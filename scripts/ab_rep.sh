#!/bin/bash
# GPU box: repeated C2 / C3 lines, default vs one knob set (VAR=VAL), interleaved
#   VAR=MR_NO_DET_FUSE VAL=1 REPS=3 scripts/ab_rep.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in $(seq ${REPS:-3}); do
  for mode in def knob; do
    for cfg in ${CFGS:-c2 c3}; do
      if [ $mode = knob ]; then export $VAR=$VAL; else unset $VAR; fi
      timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-traffic > gpurun_out/abr_${cfg}_${mode}_$r.json 2> gpurun_out/abr_${cfg}_${mode}_$r.err || { echo "$mode $cfg failed"; tail -3 gpurun_out/abr_${cfg}_${mode}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2:], d.get('windows_per_s'), d['roofline']['frac'])" gpurun_out/abr_${cfg}_${mode}_$r.json $mode $cfg $r
    done
  done
done
