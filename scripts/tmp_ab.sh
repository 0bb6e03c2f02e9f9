cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline',{});print(sys.argv[2], d['value'], d.get('windows_per_s'), d['ms_per_step'], r.get('avg_launch_us'), r.get('frac'))" "$1" "$2"; }
for rep in 1 2; do
  for e in "-" "MR_WIN_GROUP=64" "MR_WIN_GROUP=32" "MR_WIN_GROUP=64 MR_WIN_CHUNK=8"; do
    ee=$e; [ "$e" = "-" ] && ee=""
    env $ee timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --no-side --steps 8 --warmup 2 > gpurun_out/hab.json 2> gpurun_out/hab.err || { tail -5 gpurun_out/hab.err; exit 1; }
    line gpurun_out/hab.json "[$e] rep $rep"
  done
done
