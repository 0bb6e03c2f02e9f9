#!/bin/bash
# GPU box: wide-path parity tests, then the c5 line (with PMC traffic)
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_pagerank.py -k "wide or c5 or kind_compressed" -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/q_$TAG.log 2>&1; rc=$?; grep -E "PASS|FAIL|passed|failed" gpurun_out/q_$TAG.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || { tail -5 gpurun_out/c5_$TAG.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print('c5',d['value'],r['avg_launch_us'],r['frac'],r.get('traffic'))" gpurun_out/c5_$TAG.json
