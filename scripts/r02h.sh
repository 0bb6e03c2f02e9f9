#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 600 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_shard.py tests/test_gpu_rca.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-traffic > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err || { tail -3 gpurun_out/c4_$TAG.err; exit 1; }
echo "c4: $(python3 -c "import json;d=json.load(open('gpurun_out/c4_$TAG.json'));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'])")"
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu --no-traffic > gpurun_out/c2_$TAG.json 2> gpurun_out/c2_$TAG.err || { tail -3 gpurun_out/c2_$TAG.err; exit 1; }
echo "c2: $(python3 -c "import json;d=json.load(open('gpurun_out/c2_$TAG.json'));r=d['roofline'];print(d['value'],d['windows_per_s'],r['avg_launch_us'],r['frac'])")"
