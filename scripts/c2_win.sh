#!/bin/bash
# GPU box: one C2 window at W=1 -- per-phase wall times (MR_WIN_TIMING) and the kernel table
#   scripts/c2_win.sh TAG
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MR_WIN_TIMING=1 timeout -k 10 300 python3 scripts/prof_window.py 6 > gpurun_out/c2w_$TAG.log 2>&1 || { tail -5 gpurun_out/c2w_$TAG.log; exit 1; }
grep -E "window|slo" gpurun_out/c2w_$TAG.log | tail -8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2k_$TAG -o run --output-format csv -- python3 scripts/prof_window.py 6 > gpurun_out/c2k_$TAG.log 2>&1 || { tail -5 gpurun_out/c2k_$TAG.log; exit 1; }
f=$(find gpurun_out/c2k_$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"kernels: {sum(int(r['Calls']) for r in rows)} launches, {tot/1e6:.2f} ms total (7 windows + slo)")
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:26]:
    print(f'{r["Name"][:60]:60s} n={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:8.2f} tot_ms={float(r["TotalDurationNs"])/1e6:7.2f}')
PY
