cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline',{});print(sys.argv[2], d['value'], d.get('windows_per_s'), d['ms_per_step'], r.get('avg_launch_us'), r.get('frac'))" "$1" "$2"; }
for rep in 1 2; do
  for lib in ${LIBS:-abl/lib_r4.so abl/lib_r8.so}; do
    MR_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --no-side --steps 8 --warmup 2 > gpurun_out/hab.json 2> gpurun_out/hab.err || { tail -5 gpurun_out/hab.err; exit 1; }
    line gpurun_out/hab.json "[$lib] rep $rep"
  done
done
for lib in ${LIBS:-abl/lib_r4.so abl/lib_r8.so}; do
  MR_LIB_PATH=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/isoab -o run --output-format csv -- python3 scripts/chunk_iso.py 10 4 > gpurun_out/isoab.log 2>&1 || { tail -5 gpurun_out/isoab.log; exit 1; }
  echo "[$lib] $(grep 'host ms' gpurun_out/isoab.log)"
  python3 scripts/win1_trace.py --analyze $(find gpurun_out/isoab -name '*kernel_trace.csv' | head -1) | tail -1 | cut -c1-400
  rm -rf gpurun_out/isoab
done
