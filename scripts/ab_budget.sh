#!/bin/bash
# GPU box: C2 / C3 bench lines under k_tr_a block budgets (MR_TR_BUDGET)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in ${BS:-0 1 2 4}; do
  for cfg in c2 c3; do
    MR_TR_BUDGET=$b timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-traffic > gpurun_out/bud_${cfg}_$b.json 2> gpurun_out/bud_${cfg}_$b.err || { echo "b=$b $cfg failed"; tail -3 gpurun_out/bud_${cfg}_$b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['value'], d.get('windows_per_s'), r['avg_launch_us'], r['frac'])" gpurun_out/bud_${cfg}_$b.json $b $cfg
  done
done
