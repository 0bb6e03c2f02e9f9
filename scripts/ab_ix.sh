#!/bin/bash
# GPU box: k_ix_stats duration vs its block cap (MR_IX_BLOCKS) on the C2 window.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 1024 512 256 128; do
  MR_IX_BLOCKS=$b timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ix_$b -o run --output-format csv \
      -- python3 scripts/prof_window.py 4 > gpurun_out/ix_$b.log 2>&1 || exit 1
  f=$(find gpurun_out/ix_$b -name '*kernel_stats.csv' | head -1)
  echo "== $b"; python3 scripts/kstats.py "$f" 40 | grep -E "k_ix_stats|k_fx_a|build_nodes|k_node"
done
