cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MR_LO_TIMING=1 timeout -k 10 300 python3 scripts/chunk_iso.py 2 1 > gpurun_out/tim_1.log 2>&1 || { tail -5 gpurun_out/tim_1.log; exit 1; }
tail -9 gpurun_out/tim_1.log
MR_LO_TIMING=1 timeout -k 10 300 python3 scripts/chunk_iso.py 2 4 > gpurun_out/tim_4.log 2>&1 || { tail -5 gpurun_out/tim_4.log; exit 1; }
tail -10 gpurun_out/tim_4.log
