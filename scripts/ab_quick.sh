#!/bin/bash
# A/B: new short-tile walk (default build) -- pagerank GPU tests, c4 and c2 bench lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_rca.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/q_ab1.log 2>&1; rc=$?; tail -3 gpurun_out/q_ab1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --config c4 --steps 5 --warmup 1 --no-traffic --no-cpu > gpurun_out/c4_ab1.json 2> gpurun_out/c4_ab1.err || { tail -5 gpurun_out/c4_ab1.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c4_ab1.json'));r=d['roofline'];print('c4',d['value'],r['avg_launch_us'],r['frac'])"
timeout -k 10 300 python3 bench.py --no-traffic --no-cpu > gpurun_out/c2_ab1.json 2> gpurun_out/c2_ab1.err || { tail -5 gpurun_out/c2_ab1.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c2_ab1.json'));r=d['roofline'];print('c2',d['value'],d.get('windows_per_s'),r['avg_launch_us'],r['frac'])"
