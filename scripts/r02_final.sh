#!/bin/bash
# GPU box: the round's evidence -- full -m gpu suite, smoke, default bench line (with PMC traffic
# and CPU baseline), rocprofv3 kernel stats of the default bench command, c3 / c4 / sweep / ingest lines
#   scripts/r02_final.sh TAG
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
echo "smoke: $(tail -1 gpurun_out/smoke_$TAG.log)"
timeout -k 10 600 python3 bench.py > gpurun_out/c2_$TAG.json 2> gpurun_out/c2_$TAG.err || { tail -5 gpurun_out/c2_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c2_$TAG.json'));r=d['roofline'];print('c2', d['value'], d['windows_per_s'], r['avg_launch_us'], r['frac'], r['traffic'], d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pc2_$TAG -o run --output-format csv \
    -- python3 bench.py --no-traffic --no-cpu --steps 10 --warmup 2 > gpurun_out/pc2_$TAG.json 2> gpurun_out/pc2_$TAG.err || { echo "rocprof failed"; exit 1; }
echo "rocprof ok"
timeout -k 10 400 python3 bench.py --config c3 --no-traffic > gpurun_out/c3_$TAG.json 2> gpurun_out/c3_$TAG.err || { tail -5 gpurun_out/c3_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c3_$TAG.json'));r=d['roofline'];print('c3', d['value'], d['windows_per_s'], r['avg_launch_us'], r['frac'])"
timeout -k 10 500 python3 bench.py --config c4 --steps 5 --warmup 1 > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err || { tail -5 gpurun_out/c4_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c4_$TAG.json'));r=d['roofline'];print('c4', d['value'], r['avg_launch_us'], r['frac'], r['traffic'])"
timeout -k 10 300 python3 bench.py --config sweep > gpurun_out/sweep_$TAG.json 2> gpurun_out/sweep_$TAG.err || { tail -5 gpurun_out/sweep_$TAG.err; exit 1; }
timeout -k 10 300 python3 bench.py --config ingest > gpurun_out/ingest_$TAG.json 2> gpurun_out/ingest_$TAG.err || { tail -5 gpurun_out/ingest_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/sweep_$TAG.json'));e=json.load(open('gpurun_out/ingest_$TAG.json'));print('sweep', d['value'], d['window_loop']['speedup_of_sweep'], d['sliding']['windows_per_s'], 'ingest', e['value'], e['cpu_baseline']['value'])"
