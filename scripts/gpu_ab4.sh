cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q_ab4.log 2>&1; rc=$?; tail -5 gpurun_out/q_ab4.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_env.sh h "MR_TR_HOT=0" "" "MR_TR_HOT=0" "" "MR_TR_HOT=4"
