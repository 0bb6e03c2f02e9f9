#!/bin/bash
# GPU box: C2 / C3 bench lines under (hardware queues, auxiliary streams) pairs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for qs in ${PAIRS:-4:4 8:7 8:8 16:12}; do
  q=${qs%:*}; s=${qs#*:}
  for cfg in c2 c3; do
    GPU_MAX_HW_QUEUES=$q MR_WIN_STREAMS=$s timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-traffic > gpurun_out/hq_${cfg}_$q_$s.json 2> gpurun_out/hq_${cfg}_$q_$s.err || { echo "q=$q s=$s $cfg failed"; tail -3 gpurun_out/hq_${cfg}_$q_$s.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d.get('windows_per_s'), d['roofline']['avg_launch_us'])" gpurun_out/hq_${cfg}_$q_$s.json "$cfg q=$q s=$s"
  done
done
