#!/bin/bash
# GPU box: A/B of two builds of the library (MR_LIB_PATH: microrank_amd/libmicrorank_hip_ab.so = the
# previous build, built beside the tree beforehand) -- parity tests, the c2 / c3 lines interleaved
# twice, then one WRITE_SIZE pass over a c2 call (per-kernel bytes, scripts/pmc_kernels.py)
#   scripts/ab_lib.sh TAG "TEST FILES" KERNEL_REGEX
TAG=$1; TESTS=$2; KRE=${3:-k_tr_a}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 240 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
AB_VAR=MR_LIB_PATH AB_VALS="$PWD/microrank_amd/libmicrorank_hip_ab.so $PWD/microrank_amd/libmicrorank_hip.so" bash scripts/r04.sh $TAG "c2ab c3ab" || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_$TAG -o run --output-format csv -- python3 bench.py --no-traffic --no-cpu --no-side --steps 1 --warmup 0 --c2-distinct 64 > gpurun_out/pmcw_$TAG.json 2> gpurun_out/pmcw_$TAG.err || exit 1
python3 scripts/pmc_kernels.py gpurun_out/pmcw_$TAG 40 > gpurun_out/pmc_$TAG.txt && rm -rf gpurun_out/pmcw_$TAG && grep -E "$KRE" gpurun_out/pmc_$TAG.txt
