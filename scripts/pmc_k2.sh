#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a K2-only workload.
#   scripts/pmc_k2.sh TAG "cmd args"   e.g. "scripts/prof_pagerank.py 1000 200000 3"
TAG=$1; CMD=${2:-scripts/prof_pagerank.py 1000 200000 3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 $CMD \
      > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  echo "pass $i ok"
done
