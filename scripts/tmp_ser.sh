cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 bash scripts/prof_bench.sh ser --no-cpu --no-side --steps 3 --warmup 1 --c2-distinct 64 || exit 1
