#!/bin/bash
# GPU box: bench lines (C2 default with PMC traffic, C4 sharded at 1 GPU), MR_WIN_TIMING phase
# report of the C2 window, rocprofv3 kernel stats of both.   scripts/gpu_snapshot.sh TAG
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err
rc=$?; echo "bench c2 rc=$rc"; cat gpurun_out/b_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/b_$TAG.err; exit $rc; }
MR_WIN_TIMING=1 timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --steps 3 --warmup 1 > /dev/null 2> gpurun_out/wt_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python3 scripts/prof_window.py 6 > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
timeout -k 10 500 python3 bench.py --config c4 --steps 5 --warmup 1 > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err
rc=$?; echo "bench c4 rc=$rc"; cat gpurun_out/c4_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/c4_$TAG.err; exit $rc; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4_$TAG -o run --output-format csv \
    -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-traffic > gpurun_out/prof4_$TAG.log 2>&1 || { tail -5 gpurun_out/prof4_$TAG.log; exit 1; }
for d in prof_$TAG prof4_$TAG; do
  f=$(find gpurun_out/$d -name '*kernel_stats.csv' | head -1); echo "== $d"; python3 scripts/kstats.py "$f" 14
done
