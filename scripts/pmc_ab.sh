#!/bin/bash
# PMC pass 1/2 counters of k_tr_a under an environment setting: scripts/pmc_ab.sh TAG "ENV"
TAG=$1; E=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  env $E timeout -s KILL 200 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- \
      python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu --no-traffic > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?
  python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_$i k_tr_a > gpurun_out/pmc_${TAG}_$i.txt 2>&1
  cat gpurun_out/pmc_${TAG}_$i.txt
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_${TAG}_$i.log; exit $rc; }
done
