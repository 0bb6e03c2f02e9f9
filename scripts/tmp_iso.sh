cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MR_PR_HOST_TIMING=1 timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --no-side --steps 3 --warmup 1 > gpurun_out/ht.json 2> gpurun_out/ht.err || { tail -5 gpurun_out/ht.err; exit 1; }
grep "pagerank host ng=256" gpurun_out/ht.err | tail -6
