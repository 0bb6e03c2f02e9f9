#!/bin/bash
# GPU box: kernel-trace stats of the C2 window bench (and stamps) for quick A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-x}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2p_$TAG -o run --output-format csv -- python3 bench.py --no-traffic --steps 5 --warmup 2 > gpurun_out/c2p_$TAG.log 2>&1 || { tail -5 gpurun_out/c2p_$TAG.log; exit 1; }
f=$(find gpurun_out/c2p_$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:60]:60s} n={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1e3:8.2f} tot_ms={float(r["TotalDurationNs"])/1e6:8.2f}')
PY
MR_FX_STAMP=1 timeout -k 10 300 python3 bench.py --no-traffic --steps 2 --warmup 1 > /dev/null 2> gpurun_out/c2s_$TAG.err || exit 1
grep stamp gpurun_out/c2s_$TAG.err | tail -2
