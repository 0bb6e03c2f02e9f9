#!/bin/bash
# GPU box: pagerank/rca parity tests, then C2 / C3 bench lines under k_fx_b block sizes (MR_FB_W)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_rca.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_fbw.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t_fbw.log; [ $rc -eq 0 ] || exit $rc
for b in ${BS:-16 0}; do
  for cfg in c2 c3; do
    MR_FB_W=$b timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-traffic > gpurun_out/fbw_${cfg}_$b.json 2> gpurun_out/fbw_${cfg}_$b.err || { echo "b=$b $cfg failed"; tail -3 gpurun_out/fbw_${cfg}_$b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['value'], d.get('windows_per_s'), r['avg_launch_us'], r['frac'])" gpurun_out/fbw_${cfg}_$b.json $b $cfg
  done
done
