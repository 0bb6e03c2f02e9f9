#!/bin/bash
# GPU box: HBM bytes per kernel of the C5 iteration (FETCH_SIZE x2 on gfx950, WRITE_SIZE; one
# rocprofv3 pass each) -> gpurun_out/pmc_c5_TAG_*.txt
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $ctr -d gpurun_out/pmc_c5_${TAG}_$i -o run --output-format csv -- \
      python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu --no-traffic > gpurun_out/pmc_c5_${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i ($ctr) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_c5_${TAG}_$i.log; exit $rc; }
  for k in k_tr_a k_cold_ops k_cold_trace k_fx_b; do
    echo -n "$k "; python3 scripts/pmc_summary.py gpurun_out/pmc_c5_${TAG}_$i $k
  done | tee gpurun_out/pmc_c5_${TAG}_$i.txt
  find gpurun_out/pmc_c5_${TAG}_$i -name '*.csv' -size +20M -delete
done
