#!/bin/bash
# GPU box: pagerank/shard/rca parity tests with the default fused kernel, then C4 and C2 benches
# for each kernel in KERNELS (MR_FX_KERNEL: tr / wv / v1).   scripts/ab_tr.sh TAG
TAG=${1:-x}; KERNELS=${KERNELS:-"tr wv"}; TESTS=${TESTS:-1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "$TESTS" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_shard.py tests/test_gpu_rca.py -m gpu -x -q \
      --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for k in $KERNELS; do
  export MR_FX_KERNEL=$k
  timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-traffic > gpurun_out/c4_${TAG}_$k.json \
      2> gpurun_out/c4_${TAG}_$k.err || { tail -3 gpurun_out/c4_${TAG}_$k.err; exit 1; }
  echo "c4 $k: $(python3 -c "import json;d=json.load(open('gpurun_out/c4_${TAG}_$k.json'));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'])")"
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu --no-traffic > gpurun_out/c2_${TAG}_$k.json \
      2> gpurun_out/c2_${TAG}_$k.err || { tail -3 gpurun_out/c2_${TAG}_$k.err; exit 1; }
  echo "c2 $k: $(python3 -c "import json;d=json.load(open('gpurun_out/c2_${TAG}_$k.json'));r=d['roofline'];print(d['value'],d['windows_per_s'],r['avg_launch_us'],r['frac'])")"
done
if [ -n "$PROF" ]; then
  unset MR_FX_KERNEL
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4p_${TAG} -o run --output-format csv -- python3 bench.py \
      --config c4 --steps 2 --warmup 1 --no-cpu --no-traffic > gpurun_out/c4p_${TAG}.log 2>&1 || { echo "c4 prof failed"; exit 1; }
  f=$(find gpurun_out/c4p_${TAG} -name '*kernel_stats.csv' | head -1)
  echo "== c4 kernels"; python3 scripts/kstats.py "$f" 10
fi
