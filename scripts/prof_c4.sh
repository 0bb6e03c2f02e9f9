#!/bin/bash
# rocprofv3 kernel stats of the c4 bench under an environment setting: scripts/prof_c4.sh TAG "ENV"
TAG=$1; E=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pk_$TAG -o run --output-format csv \
    -- python3 bench.py --config ${CFG:-c4} --steps 3 --warmup 1 --no-traffic --no-cpu > gpurun_out/pk_$TAG.json 2> gpurun_out/pk_$TAG.err || { tail -5 gpurun_out/pk_$TAG.err; exit 1; }
python3 scripts/kstats.py $(ls gpurun_out/pk_$TAG/*kernel_stats.csv gpurun_out/pk_$TAG/*/*kernel_stats.csv 2>/dev/null | head -1) 10
