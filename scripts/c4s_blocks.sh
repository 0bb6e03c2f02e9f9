#!/bin/bash
# GPU box: C4 rank-0-of-8 share with k_tr_a's block count forced (MR_TR_BLOCKS) -> one line each
#   scripts/c4s_blocks.sh TAG "0 192 128 96"      (0: the default plan)
TAG=${1:-x}; LIST=${2:-"0 192 128"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for nb in $LIST; do
  E=""; [ "$nb" != 0 ] && E="MR_TR_BLOCKS=$nb"
  timeout -k 10 300 env $E python3 bench.py --config c4 --shard-of 8 --no-cpu --no-traffic --steps 20 --warmup 3 \
      > gpurun_out/c4s_${TAG}_$nb.json 2> gpurun_out/c4s_${TAG}_$nb.err || { tail -5 gpurun_out/c4s_${TAG}_$nb.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print('blocks', sys.argv[2], d['value'], d['ms_per_step'], r.get('avg_launch_us'))" gpurun_out/c4s_${TAG}_$nb.json "$nb"
done
