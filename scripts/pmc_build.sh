#!/bin/bash
# HBM traffic per kernel of the C5 rank-share span build (+ its PageRank):
#   scripts/pmc_build.sh TAG   (GPU box; one rocprofv3 --pmc run per counter, summaries to gpurun_out/)
TAG=${1:-b}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr -d gpurun_out/pmcb_${TAG}_$ctr -o run --output-format csv -- \
      python3 bench.py --config c5 --from-spans --shard-of 8 --steps 1 --warmup 1 --no-cpu --no-traffic \
      > gpurun_out/pmcb_${TAG}_$ctr.log 2>&1
  rc=$?
  echo "$ctr rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pmcb_${TAG}_$ctr.log; exit $rc; }
  python3 scripts/pmc_kernels.py gpurun_out/pmcb_${TAG}_$ctr 25 > gpurun_out/pmcb_${TAG}_$ctr.txt
  head -14 gpurun_out/pmcb_${TAG}_$ctr.txt
done
