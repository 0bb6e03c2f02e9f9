#!/bin/bash
# GPU box: C2 / C3 bench lines for windows per mr_windows_batch call (--streams) x MR_WIN_CHUNK
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for s in ${SS:-64 256}; do
  for ch in ${CHS:-4}; do
    for cfg in ${CFGS:-c2 c3}; do
      MR_WIN_CHUNK=$ch timeout -k 10 300 python3 bench.py --config $cfg --streams $s --no-cpu --no-traffic > gpurun_out/abc_${cfg}_${s}_$ch.json 2> gpurun_out/abc_${cfg}_${s}_$ch.err || { echo "$s $ch $cfg failed"; tail -3 gpurun_out/abc_${cfg}_${s}_$ch.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2:], d['value'], d.get('windows_per_s'), r['avg_launch_us'], r['frac'])" gpurun_out/abc_${cfg}_${s}_$ch.json $s $ch $cfg
    done
  done
done
