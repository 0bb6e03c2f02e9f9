#!/bin/bash
# GPU box: parity suites of the iteration (pagerank, shard, rca) then c4 / c2 / c3 lines
#   scripts/gpu_check.sh TAG
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_shard.py tests/test_gpu_rca.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/q_$TAG.log; [ $rc -eq 0 ] || exit $rc
for c in c4 c2 c3; do
  timeout -k 10 400 python3 bench.py --config $c --no-traffic --no-cpu > gpurun_out/${c}_$TAG.json 2> gpurun_out/${c}_$TAG.err || { tail -5 gpurun_out/${c}_$TAG.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['value'],d.get('windows_per_s'),r['avg_launch_us'],r['frac'])" gpurun_out/${c}_$TAG.json $c
done
