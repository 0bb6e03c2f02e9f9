cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_rca.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_fill.log 2>&1; rc=$?; tail -2 gpurun_out/t_fill.log; [ $rc -eq 0 ] || exit $rc
AB_VAR=MR_LIB_PATH AB_VALS="$PWD/microrank_amd/libmicrorank_hip_ab.so $PWD/microrank_amd/libmicrorank_hip.so" bash scripts/r04.sh fill "c2ab c3ab" || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf -o run --output-format csv -- python3 bench.py --no-traffic --no-cpu --no-side --steps 1 --warmup 0 --c2-distinct 64 > gpurun_out/pmcf.json 2> gpurun_out/pmcf.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o run --output-format csv -- python3 bench.py --no-traffic --no-cpu --no-side --steps 1 --warmup 0 --c2-distinct 64 > gpurun_out/pmcw.json 2> gpurun_out/pmcw.err || exit 1
python3 scripts/pmc_kernels.py gpurun_out/pmcf 40 > gpurun_out/pmc_c2.txt && python3 scripts/pmc_kernels.py gpurun_out/pmcw 40 >> gpurun_out/pmc_c2.txt && rm -rf gpurun_out/pmcf gpurun_out/pmcw
