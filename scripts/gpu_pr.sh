#!/bin/bash
# GPU box: pagerank + shard parity suites, then c4 and c4 --from-spans lines
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_shard.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/q_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/q_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config c4 --steps 5 --warmup 1 --no-traffic --no-cpu > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err || { tail -5 gpurun_out/c4_$TAG.err; exit 1; }
timeout -k 10 400 python3 bench.py --config c4 --from-spans --steps 5 --warmup 1 --no-traffic --no-cpu > gpurun_out/c4s_$TAG.json 2> gpurun_out/c4s_$TAG.err || { tail -5 gpurun_out/c4s_$TAG.err; exit 1; }
for c in c4 c4s; do python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['value'],d['ms_per_step'],d.get('build_ms'),r['avg_launch_us'],r['frac'])" gpurun_out/${c}_$TAG.json $c; done
