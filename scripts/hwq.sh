#!/bin/bash
# GPU box: C2 / C3 bench lines under HIP hardware-queue counts (GPU_MAX_HW_QUEUES)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for q in ${QS:-4 8 16}; do
  for cfg in c2 c3; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-traffic > gpurun_out/hwq_${cfg}_$q.json 2> gpurun_out/hwq_${cfg}_$q.err || { echo "q=$q $cfg failed"; tail -3 gpurun_out/hwq_${cfg}_$q.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d.get('windows_per_s'), d['roofline']['frac'])" gpurun_out/hwq_${cfg}_$q.json $q $cfg
  done
done
