#!/bin/bash
# GPU box: round-2 evidence -- bench lines (c2 default incl. PMC traffic + CPU baseline, c3, c4 incl.
# traffic, c4 from spans, c5), rocprof kernel tables (c2 bench command, c4), k_tr_a PMC passes,
# the RCCL 1-rank all-reduce latency.  Outputs under gpurun_out/r02/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02; mkdir -p $O
set -o pipefail
run() { local name=$1; shift; echo "== $name"; timeout -k 10 ${T:-600} "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed rc=$?"; tail -5 $O/$name.err; return 1; }; tail -c 600 $O/$name.json; echo; }
PART=${1:-a}
if [ $PART = a ]; then
run bench_c2 python3 bench.py || exit 1
T=500 run bench_c3 python3 bench.py --config c3 --no-cpu --no-traffic || exit 1
T=700 run bench_c4 python3 bench.py --config c4 || exit 1
timeout -k 10 120 python3 scripts/rccl_latency.py > $O/rccl.json 2> $O/rccl.err; cat $O/rccl.json
exit 0
fi
if [ $PART = b ]; then
T=500 run bench_c4_spans python3 bench.py --config c4 --from-spans --steps 3 --warmup 1 --no-cpu --no-traffic || exit 1
T=600 run bench_c5 python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu --no-traffic || exit 1
exit 0
fi
for cfg in c2 c4; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu --no-traffic > $O/prof_$cfg.log 2>&1 || { echo "prof $cfg failed"; exit 1; }
  f=$(find $O/prof_$cfg -name "*kernel_stats.csv" | head -1); cp $f $O/${cfg}_kernel_stats.csv
done
TAG=r02 scripts/pmc_c4.sh r02 k_tr_a > $O/pmc_c4.txt 2>&1; cp gpurun_out/pmc_r02_*.txt $O/ 2>/dev/null
echo done
