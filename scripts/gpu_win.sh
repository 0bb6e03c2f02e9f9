#!/bin/bash
# GPU box: window parity suite (rca + graph build), then c2 / c3 A/B of an environment setting
TAG=${1:-x}; E=${2:-MR_NO_IXB=1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rca.py tests/test_gpu_graph_build.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/q_$TAG.log; [ $rc -eq 0 ] || exit $rc
CFG=c2 EXTRA="--steps 10 --warmup 2" bash scripts/ab_env.sh ${TAG}2 "" "$E" "" "$E" && CFG=c3 EXTRA="--steps 10 --warmup 2" bash scripts/ab_env.sh ${TAG}3 "" "$E" "" "$E"
