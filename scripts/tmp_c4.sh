cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/prof_bench.sh c4s8 --config c4 --no-cpu --shard-of 8 --steps 10 --warmup 2 || exit 1
bash scripts/prof_bench.sh c5 --config c5 --no-cpu --steps 5 --warmup 1 || exit 1
