#!/bin/bash
# GPU box: single-window latency (W=1) of the C2 / C3 bench, with MR_WIN_TIMING phase marks
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in c2 c3; do
  timeout -k 10 300 python3 bench.py --config $cfg --streams 1 --c3-windows 1 --steps 20 --warmup 3 --no-cpu --no-traffic > gpurun_out/w1_$cfg.json 2> gpurun_out/w1_$cfg.err || { tail -3 gpurun_out/w1_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('windows_per_s'))" gpurun_out/w1_$cfg.json $cfg
  MR_WIN_TIMING=1 timeout -k 10 300 python3 bench.py --config $cfg --streams 1 --c3-windows 1 --steps 3 --warmup 2 --no-cpu --no-traffic > /dev/null 2> gpurun_out/w1t_$cfg.err || exit 1
  tail -12 gpurun_out/w1t_$cfg.err
done
