#!/bin/bash
# GPU box: kernel table of the C5 bench (wide fused path)   scripts/c5_prof.sh TAG [extra bench args]
TAG=${1:-x}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/c5p_$TAG -o run --output-format csv -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu --no-traffic "$@" > gpurun_out/c5p_$TAG.log 2>&1 || { tail -5 gpurun_out/c5p_$TAG.log; exit 1; }
tail -1 gpurun_out/c5p_$TAG.log
f=$(find gpurun_out/c5p_$TAG -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/c5p_${TAG}_kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"kernels: {sum(int(r['Calls']) for r in rows)} launches, {tot/1e6:.2f} ms total")
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:30]:
    print(f'{r["Name"][:60]:60s} n={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f} tot_ms={float(r["TotalDurationNs"])/1e6:8.2f}')
PY
