#!/bin/bash
# PMC passes over the C2 window-group iteration kernel (one rocprofv3 run per counter group, <= 8 SQ
# each): scripts/pmc_c2.sh TAG [kernel-pattern] [extra env assignments...]   (GPU box)
#   BARGS: the bench arguments (default the C2 line on 16 distinct windows; C3: "--config c3 --steps 1 --warmup 1")
TAG=${1:-c2}; PAT=${2:-k_tr_a}; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for kv in "$@"; do export "$kv"; done
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- \
      python3 bench.py ${BARGS:---c2-distinct 16 --steps 1 --warmup 1} --no-cpu --no-traffic --no-side \
      > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_$i $PAT > gpurun_out/pmc_${TAG}_$i.txt 2>&1
  cat gpurun_out/pmc_${TAG}_$i.txt
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_${TAG}_$i.log; exit $rc; }
done
