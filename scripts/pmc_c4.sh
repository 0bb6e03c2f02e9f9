#!/bin/bash
# PMC passes over the C4 iteration kernel (one rocprofv3 run per counter group, <= 8 SQ each).
#   scripts/pmc_c4.sh TAG [kernel-pattern] [config]   (GPU box; summaries to gpurun_out/pmc_TAG_*.txt)
TAG=${1:-c4}; PAT=${2:-k_tr_a}; CFG=${3:-c4}; OPS=${OPS:-10000}; TRACES=${TRACES:-10000000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- \
      python3 bench.py --config $CFG --c4-ops $OPS --c4-traces $TRACES --steps 1 --warmup 1 --no-cpu --no-traffic \
      > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_$i $PAT > gpurun_out/pmc_${TAG}_$i.txt 2>&1
  cat gpurun_out/pmc_${TAG}_$i.txt
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_${TAG}_$i.log; exit $rc; }
done
