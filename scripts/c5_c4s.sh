#!/bin/bash
# GPU box: C5 (100k ops / 100M traces fp32) and C4 from span shards bench lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 600 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || { tail -5 gpurun_out/c5_$TAG.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print('c5', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r.get('traffic'))" gpurun_out/c5_$TAG.json
timeout -k 10 600 python3 bench.py --config c4 --from-spans --steps 3 --warmup 1 --no-cpu --no-traffic > gpurun_out/c4s_$TAG.json 2> gpurun_out/c4s_$TAG.err || { tail -5 gpurun_out/c4s_$TAG.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print('c4s', d['value'], d['ms_per_step'], d.get('build_ms'), r['frac'])" gpurun_out/c4s_$TAG.json
