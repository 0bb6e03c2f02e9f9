#!/bin/bash
# GPU box: rocprofv3 kernel table of one bench command   scripts/prof.sh TAG [bench args...]
# prints the top kernels and the summed kernel time per window (windows = k_ix_detect launches)
TAG=${1:-x}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_$TAG -o run --output-format csv -- python3 bench.py --no-traffic --no-cpu "$@" > gpurun_out/p_$TAG.log 2>&1 || { tail -5 gpurun_out/p_$TAG.log; exit 1; }
grep -h '"metric"' gpurun_out/p_$TAG.log | tail -1 | cut -c1-300
f=$(find gpurun_out/p_$TAG -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/p_${TAG}_kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
nw = sum(int(r["Calls"]) for r in rows if "k_ix_detect" in r["Name"]) or 1
print(f"kernels: {sum(int(r['Calls']) for r in rows)} launches, {tot/1e6:.2f} ms total, {nw} windows, "
      f"{tot/1e6/nw:.3f} ms / window, {sum(int(r['Calls']) for r in rows)/nw:.1f} launches / window")
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:45]:
    t = float(r["TotalDurationNs"])
    print(f'{r["Name"][:58]:58s} n/w={int(r["Calls"])/nw:6.2f} avg_us={float(r["AverageNs"])/1e3:8.2f} us/w={t/1e3/nw:8.2f}')
PY
