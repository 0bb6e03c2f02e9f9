cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/iso_1 -o run --output-format csv -- python3 scripts/chunk_iso.py 10 1 > gpurun_out/iso_1.log 2>&1 || { tail -5 gpurun_out/iso_1.log; exit 1; }
grep "host ms" gpurun_out/iso_1.log
timeout -k 10 300 python3 scripts/chunk_iso.py 20 1 2>&1 | grep "host ms"
python3 scripts/call_timeline.py $(find gpurun_out/iso_1 -name '*kernel_trace.csv' | head -1) > gpurun_out/iso_1_timeline.txt
cat gpurun_out/iso_1_timeline.txt | head -120
