#!/bin/bash
# GPU box: mr_windows_batch host phase timers (MR_WIN_PHASES=1) for c2 and c3 bench calls
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in c2 c3; do
  MR_WIN_PHASES=1 timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 > gpurun_out/ph_${TAG}_$c.json 2> gpurun_out/ph_${TAG}_$c.err || exit $?
  tail -4 gpurun_out/ph_${TAG}_$c.err
done
