cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rca.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c2_windows or layout_order or c3_window or standalone or driver" > gpurun_out/t_lo3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_lo3.log; [ $rc -eq 0 ] || exit $rc
MR_LO_TIMING=1 timeout -k 10 300 python3 scripts/chunk_iso.py 1 4 > gpurun_out/tim_4.log 2>&1 || { tail -5 gpurun_out/tim_4.log; exit 1; }
tail -14 gpurun_out/tim_4.log
