cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/all_c2.json 2> gpurun_out/all_c2.err || { tail -5 gpurun_out/all_c2.err; exit 1; }
cut -c1-3000 gpurun_out/all_c2.json
for c in c3 c4 c5; do
  timeout -k 10 400 python3 bench.py --config $c --no-cpu > gpurun_out/all_$c.json 2> gpurun_out/all_$c.err || { tail -5 gpurun_out/all_$c.err; exit 1; }
  cut -c1-1500 gpurun_out/all_$c.json
done
