cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_full.log; [ $rc -eq 0 ] || exit $rc
echo "W1 $(timeout -k 10 300 python3 scripts/chunk_iso.py 30 1 2>&1 | grep 'host ms')"
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline',{});print(sys.argv[2], d['value'], d.get('windows_per_s'), d['ms_per_step'], r.get('avg_launch_us'), r.get('frac'), d.get('window_ms',{}).get('median'))" "$1" "$2"; }
for c in c2 c3 c4; do
timeout -k 10 400 python3 bench.py --config $c --no-traffic --no-cpu --steps 8 --warmup 2 --no-c4-leg > gpurun_out/hab_$c.json 2> gpurun_out/hab.err || { tail -5 gpurun_out/hab.err; exit 1; }
line gpurun_out/hab_$c.json $c
done
