#!/bin/bash
# GPU box: GPU tests, then the C4 iteration at the given op counts with phase stamps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_probe.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_probe.log; [ $rc -eq 0 ] || exit $rc
fi
for n in ${OPS:-10000}; do
  timeout -k 10 300 python3 bench.py --config c4 --c4-ops $n --steps 2 --warmup 1 > gpurun_out/p_$n.json 2> gpurun_out/p_$n.err || { tail -5 gpurun_out/p_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/p_$n.json'));print($n, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
  MR_FX_STAMP=1 timeout -k 10 300 python3 bench.py --config c4 --c4-ops $n --steps 1 --warmup 1 > /dev/null 2> gpurun_out/s_$n.err || { tail -5 gpurun_out/s_$n.err; exit 1; }
  grep stamp gpurun_out/s_$n.err | tail -1
done
for tt in $C2; do
  MR_TT=$tt timeout -k 10 300 python3 bench.py --no-traffic > gpurun_out/b_probe.json 2> gpurun_out/b_probe.err || { tail -5 gpurun_out/b_probe.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b_probe.json'));print('C2 TT=$tt', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
