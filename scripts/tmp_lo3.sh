cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rca.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c2_windows or layout_order or c3_window or standalone or fast_paths or driver" > gpurun_out/t_lo3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t_lo3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/iso_4 -o run --output-format csv -- python3 scripts/chunk_iso.py 10 4 > gpurun_out/iso_4.log 2>&1 || { tail -5 gpurun_out/iso_4.log; exit 1; }
grep "host ms" gpurun_out/iso_4.log
python3 scripts/win1_trace.py --analyze $(find gpurun_out/iso_4 -name '*kernel_trace.csv' | head -1) | tail -2
bash scripts/prof_bench.sh lo3 --no-cpu --no-side --steps 10 --warmup 2 || exit 1
