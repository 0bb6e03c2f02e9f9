#!/bin/bash
# GPU box: the round's evidence -- full -m gpu suite, smoke, default bench line (with PMC traffic
# and CPU baseline), rocprofv3 kernel stats of the default bench command, c3 / c4 / c5 / sweep /
# ingest / dropin lines.
#   scripts/round_final.sh TAG [stages]   (stages: t s c2 prof c3 c4 c5 c5s sweep ingest dropin; default all)
TAG=${1:-x}
STAGES=${2:-"t s c2 prof c3 c4 c5 c5s sweep ingest dropin"}
has() { [[ " $STAGES " == *" $1 "* ]]; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if has t; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if has s; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
  echo "smoke: $(tail -1 gpurun_out/smoke_$TAG.log)"
fi
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline',{});print(sys.argv[2], d['value'], d.get('windows_per_s'), r.get('avg_launch_us'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), d.get('window_ms'))" "$1" "$2"; }
if has c2; then
  timeout -k 10 900 python3 bench.py > gpurun_out/c2_$TAG.json 2> gpurun_out/c2_$TAG.err || { tail -5 gpurun_out/c2_$TAG.err; exit 1; }
  line gpurun_out/c2_$TAG.json c2
fi
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pc2_$TAG -o run --output-format csv \
      -- python3 bench.py --no-traffic --no-cpu --steps 10 --warmup 2 > gpurun_out/pc2_$TAG.json 2> gpurun_out/pc2_$TAG.err || { echo "rocprof failed"; exit 1; }
  echo "rocprof ok"
fi
if has c3; then
  timeout -k 10 400 python3 bench.py --config c3 > gpurun_out/c3_$TAG.json 2> gpurun_out/c3_$TAG.err || { tail -5 gpurun_out/c3_$TAG.err; exit 1; }
  line gpurun_out/c3_$TAG.json c3
fi
if has c4; then
  timeout -k 10 600 python3 bench.py --config c4 --steps 5 --warmup 1 > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err || { tail -5 gpurun_out/c4_$TAG.err; exit 1; }
  line gpurun_out/c4_$TAG.json c4
fi
if has c5; then
  timeout -k 10 600 python3 bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || { tail -5 gpurun_out/c5_$TAG.err; exit 1; }
  line gpurun_out/c5_$TAG.json c5
fi
if has c5s; then
  timeout -k 10 600 python3 bench.py --config c5 --from-spans --shard-of 8 --steps 3 --warmup 1 --no-traffic > gpurun_out/c5s_$TAG.json 2> gpurun_out/c5s_$TAG.err || { tail -5 gpurun_out/c5s_$TAG.err; exit 1; }
  line gpurun_out/c5s_$TAG.json c5s
fi
if has sweep; then
  timeout -k 10 300 python3 bench.py --config sweep > gpurun_out/sweep_$TAG.json 2> gpurun_out/sweep_$TAG.err || { tail -5 gpurun_out/sweep_$TAG.err; exit 1; }
  line gpurun_out/sweep_$TAG.json sweep
fi
if has ingest; then
  timeout -k 10 300 python3 bench.py --config ingest > gpurun_out/ingest_$TAG.json 2> gpurun_out/ingest_$TAG.err || { tail -5 gpurun_out/ingest_$TAG.err; exit 1; }
  line gpurun_out/ingest_$TAG.json ingest
fi
if has dropin; then
  timeout -k 10 400 python3 bench.py --config dropin > gpurun_out/dropin_$TAG.json 2> gpurun_out/dropin_$TAG.err || { tail -5 gpurun_out/dropin_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/dropin_$TAG.json'));print('dropin', d['config']['C1'], d['config']['C2'])"
fi
