cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rca.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_lo3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_lo3.log; [ $rc -eq 0 ] || exit $rc
echo "C3 W1 $(timeout -k 10 300 python3 scripts/chunk_iso.py 30 1 500 20000 2>&1 | grep 'host ms')"
echo "C2 W1 $(timeout -k 10 300 python3 scripts/chunk_iso.py 30 1 2>&1 | grep 'host ms')"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/isoab -o run --output-format csv -- python3 scripts/chunk_iso.py 10 4 > gpurun_out/isoab.log 2>&1 || { tail -5 gpurun_out/isoab.log; exit 1; }
python3 scripts/win1_trace.py --analyze $(find gpurun_out/isoab -name '*kernel_trace.csv' | head -1) | tail -1 | cut -c1-300
rm -rf gpurun_out/isoab
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline',{});print(sys.argv[2], d['value'], d.get('windows_per_s'), d['ms_per_step'], r.get('avg_launch_us'), r.get('frac'), d.get('window_ms',{}).get('median'))" "$1" "$2"; }
for rep in 1 2; do
timeout -k 10 400 python3 bench.py --no-traffic --no-cpu --steps 8 --warmup 2 --no-c4-leg > gpurun_out/hab_c2.json 2> gpurun_out/hab.err || { tail -5 gpurun_out/hab.err; exit 1; }
line gpurun_out/hab_c2.json c2
done
