#!/bin/bash
# GPU box: parity of the window builds, then A/B (MR_LIB_PATH: libmicrorank_hip_ab.so = the previous
# build) on the c2 / c3 lines, then one WRITE_SIZE pass over a c2 call
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_rca.py tests/test_gpu_shard.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_pref.log 2>&1; rc=$?; tail -2 gpurun_out/t_pref.log; [ $rc -eq 0 ] || exit $rc
AB_VAR=MR_LIB_PATH AB_VALS="$PWD/microrank_amd/libmicrorank_hip_ab.so $PWD/microrank_amd/libmicrorank_hip.so" bash scripts/r04.sh pref "c2ab c3ab" || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o run --output-format csv -- python3 bench.py --no-traffic --no-cpu --no-side --steps 1 --warmup 0 --c2-distinct 64 > gpurun_out/pmcw.json 2> gpurun_out/pmcw.err || exit 1
python3 scripts/pmc_kernels.py gpurun_out/pmcw 40 > gpurun_out/pmc_pref.txt && rm -rf gpurun_out/pmcw && grep -E "pref_apply|inv_perm|tr_place" gpurun_out/pmc_pref.txt
