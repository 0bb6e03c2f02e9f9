#!/bin/bash
# GPU box: pagerank/shard parity tests, then C4 and C2 benches with k_sg_a (default) and k_fx_a (MR_FX_V1)
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_shard.py tests/test_gpu_rca.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
for v in sg v1; do
  if [ $v = v1 ]; then export MR_FX_V1=1; fi
  timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-traffic > gpurun_out/c4_${TAG}_$v.json 2> gpurun_out/c4_${TAG}_$v.err || { echo "c4 $v failed"; tail -5 gpurun_out/c4_${TAG}_$v.err; exit 1; }
  echo "c4 $v: $(python3 -c "import json;d=json.load(open('gpurun_out/c4_${TAG}_$v.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_us'],r['frac'])")"
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu --no-traffic > gpurun_out/c2_${TAG}_$v.json 2> gpurun_out/c2_${TAG}_$v.err || { echo "c2 $v failed"; tail -5 gpurun_out/c2_${TAG}_$v.err; exit 1; }
  echo "c2 $v: $(python3 -c "import json;d=json.load(open('gpurun_out/c2_${TAG}_$v.json'));r=d['roofline'];print(d['value'],d['windows_per_s'],r['avg_launch_us'],r['frac'])")"
done
