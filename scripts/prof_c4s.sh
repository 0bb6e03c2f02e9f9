#!/bin/bash
# rocprofv3 kernel stats of the c4 --from-spans bench: scripts/prof_c4s.sh TAG "ENV"
TAG=$1; E=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pks_$TAG -o run --output-format csv \
    -- python3 bench.py --config c4 --from-spans --steps 3 --warmup 1 --no-traffic --no-cpu > gpurun_out/pks_$TAG.json 2> gpurun_out/pks_$TAG.err || { tail -5 gpurun_out/pks_$TAG.err; exit 1; }
python3 scripts/kstats.py gpurun_out/pks_$TAG/run_kernel_stats.csv 25
