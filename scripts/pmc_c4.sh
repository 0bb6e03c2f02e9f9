#!/bin/bash
# PMC passes over the C4 iteration kernels (one rocprofv3 run per counter group).
TAG=${1:-c4}; OPS=${OPS:-10000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 bench.py --config c4 --c4-ops $OPS --steps 1 --warmup 1 \
      > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  echo "pass $i ok"
  python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_$i k_fx_a
done
