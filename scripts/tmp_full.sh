cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline',{});print(sys.argv[2], d['value'], d.get('windows_per_s'), d['ms_per_step'], r.get('avg_launch_us'), r.get('frac'))" "$1" "$2"; }
timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --no-side --steps 10 --warmup 2 > gpurun_out/hab.json 2> gpurun_out/hab.err || { tail -5 gpurun_out/hab.err; exit 1; }
line gpurun_out/hab.json "c2"
