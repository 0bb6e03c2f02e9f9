#!/bin/bash
# GPU box: A/B of an environment knob on a bench config, alternating runs
#   scripts/ab_env.sh "VAR=1" [bench args...]
KNOB=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for mode in base knob; do
    if [ $mode = knob ]; then E="env $KNOB"; else E=""; fi
    $E timeout -k 10 300 python3 bench.py --no-cpu --no-traffic "$@" > gpurun_out/ab_$mode.json 2> gpurun_out/ab_$mode.err || { tail -3 gpurun_out/ab_$mode.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d.get('windows_per_s'), (d.get('window_ms') or {}).get('median'))" gpurun_out/ab_$mode.json $mode
  done
done
