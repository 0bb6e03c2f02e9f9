cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rca.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c2_windows or layout_order or c3_window or standalone or driver" > gpurun_out/t_lo3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_lo3.log; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline',{});print(sys.argv[2], d['value'], d.get('windows_per_s'), d['ms_per_step'], r.get('avg_launch_us'), r.get('frac'))" "$1" "$2"; }
for rep in 1 2; do
  for e in "-" "MR_TR_MERGE=0"; do
    ee=$e; [ "$e" = "-" ] && ee=""
    env $ee timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --no-side --steps 8 --warmup 2 > gpurun_out/hab.json 2> gpurun_out/hab.err || { tail -5 gpurun_out/hab.err; exit 1; }
    line gpurun_out/hab.json "[$e] rep $rep"
  done
done
