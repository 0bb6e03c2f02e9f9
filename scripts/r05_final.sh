#!/bin/bash
# Round-5 final evidence (GPU box): GPU tests, smoke, the default line (traffic + CPU baseline +
# side legs), c3 / c4 / c5 lines, and the kernel table of the timed C2 steps -> gpurun_out/fin_*
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/fin_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin_smoke.txt 2>&1 || { tail -5 gpurun_out/fin_smoke.txt; exit 1; }
tail -1 gpurun_out/fin_smoke.txt
timeout -k 10 900 python3 bench.py > gpurun_out/fin_c2.json 2> gpurun_out/fin_c2.err || { tail -5 gpurun_out/fin_c2.err; exit 1; }
cut -c1-400 gpurun_out/fin_c2.json
for c in c3 c4 c5; do
  timeout -k 10 600 python3 bench.py --config $c --no-cpu > gpurun_out/fin_$c.json 2> gpurun_out/fin_$c.err || { tail -5 gpurun_out/fin_$c.err; exit 1; }
  cut -c1-300 gpurun_out/fin_$c.json
done
bash scripts/prof_bench.sh fin_c2s --no-cpu --no-side --steps 10 --warmup 2 > /dev/null || exit 1
bash scripts/prof_bench.sh fin_c4s8 --config c4 --no-cpu --shard-of 8 --steps 10 --warmup 2 > /dev/null || exit 1
echo done
