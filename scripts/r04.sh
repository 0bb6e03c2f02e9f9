#!/bin/bash
# GPU box, round 4 evidence: scripts/r04.sh TAG "stages"
#   t       full -m gpu suite          s      smoke
#   c2      default bench line (c2 windows + c4_sharded leg, PMC traffic, CPU baseline)
#   pc2     rocprofv3 kernel table of the timed c2 groups only (--no-side: no latency / kind / c4 legs)
#   pc2ser  the same with one auxiliary stream and synchronous PageRank groups (kernels alone on the chip)
#   c4sp    c4 from span shards at N=1 (build inside the step)
#   pc3     rocprofv3 kernel table / trace of the timed c3 steps only
#   dropin  the drop-in line (reference driver's window body through the swapped imports)
#   w1      one C3 window per call under rocprofv3 --kernel-trace (scripts/win1_trace.py)
#   c4      c4 line (traffic, CPU baseline)       pc4   rocprofv3 kernel table of the c4 command
#   c4s8    c4 at N=1 holding rank 0's share of an 8-GPU deployment (per-rank compute at N=8)
#   pmc4    k_tr_a LDS / wait PMC passes at C4 (scripts/pmc_c4.sh)
#   segv    the rocprofv3 --kernel-trace --stats c3 command that crashed in round 3, once, with maps
#   c3 c5   c3 / c5 lines          c5s / pc5s   c5 from span shards (rank 0 of 8) / its kernel table
#   pc5     c5 kernel table          pc4s8  kernel table of c4 rank 0's share of 8
#   c3ab c2ab  AB_VAR over AB_VALS on the c3 / c2 lines (interleaved, two repeats)
#   spab    AB_VAR over AB_VALS on the span-built c4 / c5-share steps (build_ms)
#   shard   the shard tests only
TAG=${1:-x}
STAGES=${2:-"t s c2"}
has() { [[ " $STAGES " == *" $1 "* ]]; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out profiles
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline',{});print(sys.argv[2], d['value'], d.get('windows_per_s'), r.get('avg_launch_us'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), d.get('window_ms'), json.dumps(d.get('c4_sharded')))" "$1" "$2"; }
if has shard; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 240 --timeout-method thread > gpurun_out/shard_$TAG.log 2>&1
  rc=$?; echo "shard rc=$rc"; tail -3 gpurun_out/shard_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if has t; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if has s; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
  echo "smoke: $(tail -1 gpurun_out/smoke_$TAG.log)"
fi
if has c2; then
  timeout -k 10 900 python3 bench.py > gpurun_out/c2_$TAG.json 2> gpurun_out/c2_$TAG.err || { tail -5 gpurun_out/c2_$TAG.err; exit 1; }
  line gpurun_out/c2_$TAG.json c2
fi
if has pc2; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pc2_$TAG -o run --output-format csv \
      -- python3 bench.py --no-traffic --no-cpu --no-side --steps 10 --warmup 2 > gpurun_out/pc2_$TAG.json 2> gpurun_out/pc2_$TAG.err || { echo "rocprof pc2 failed"; tail -5 gpurun_out/pc2_$TAG.err; exit 1; }
  line gpurun_out/pc2_$TAG.json pc2
fi
if has pc2ser; then   # the same, one auxiliary stream and synchronous PageRank groups: kernels alone on the chip
  MR_WIN_STREAMS=1 MR_WIN_PR_SYNC=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pc2ser_$TAG -o run --output-format csv \
      -- python3 bench.py --no-traffic --no-cpu --no-side --steps 3 --warmup 1 > gpurun_out/pc2ser_$TAG.json 2> gpurun_out/pc2ser_$TAG.err || { echo "rocprof pc2ser failed"; tail -5 gpurun_out/pc2ser_$TAG.err; exit 1; }
  line gpurun_out/pc2ser_$TAG.json pc2ser
fi
if has w1; then   # one C3 window per call: host time, and the kernel trace split per call
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/w1_$TAG -o run --output-format csv \
      -- python3 scripts/win1_trace.py 20 > gpurun_out/w1_$TAG.log 2>&1 || { echo "w1 failed"; tail -5 gpurun_out/w1_$TAG.log; exit 1; }
  grep "W=1" gpurun_out/w1_$TAG.log; python3 scripts/win1_trace.py --analyze gpurun_out/w1_$TAG/run_kernel_trace.csv | tail -4
fi
if has pc3; then   # kernel table + trace of the timed c3 steps only
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pc3_$TAG -o run --output-format csv \
      -- python3 bench.py --config c3 --no-traffic --no-cpu --no-side --steps 5 --warmup 1 > gpurun_out/pc3_$TAG.json 2> gpurun_out/pc3_$TAG.err || { echo "rocprof pc3 failed"; tail -5 gpurun_out/pc3_$TAG.err; exit 1; }
  line gpurun_out/pc3_$TAG.json pc3
fi
if has dropin; then   # the reference driver's window body through the drop-in modules (C1, C2)
  timeout -k 10 600 python3 bench.py --config dropin > gpurun_out/dropin_$TAG.json 2> gpurun_out/dropin_$TAG.err || { tail -5 gpurun_out/dropin_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/dropin_$TAG.json'));c=d['config'];print('dropin C1', c['C1']['windows_per_s'], c['C1']['ms_per_window'], 'C2', c['C2']['windows_per_s'], c['C2']['ms_per_window'])"
fi
if has c4; then
  timeout -k 10 600 python3 bench.py --config c4 --steps 5 --warmup 1 > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err || { tail -5 gpurun_out/c4_$TAG.err; exit 1; }
  line gpurun_out/c4_$TAG.json c4
fi
if has pc4; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pc4_$TAG -o run --output-format csv \
      -- python3 bench.py --config c4 --no-traffic --no-cpu --steps 5 --warmup 1 > gpurun_out/pc4_$TAG.json 2> gpurun_out/pc4_$TAG.err || { echo "rocprof pc4 failed"; tail -5 gpurun_out/pc4_$TAG.err; exit 1; }
  line gpurun_out/pc4_$TAG.json pc4
fi
if has c4s8; then
  timeout -k 10 600 python3 bench.py --config c4 --shard-of 8 --steps 10 --warmup 2 --no-cpu > gpurun_out/c4s8_$TAG.json 2> gpurun_out/c4s8_$TAG.err || { tail -5 gpurun_out/c4s8_$TAG.err; exit 1; }
  line gpurun_out/c4s8_$TAG.json c4s8
fi
if has pmc4; then
  bash scripts/pmc_c4.sh $TAG k_tr_a c4 || exit 1
fi
if has segv; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/segv_$TAG -o run --output-format csv \
      -- python3 bench.py --no-traffic --config c3 --steps 3 --warmup 1 --no-cpu --dump-maps gpurun_out/maps_$TAG.txt \
      > gpurun_out/segv_$TAG.json 2> gpurun_out/segv_$TAG.err
  rc=$?; echo "segv-command rc=$rc"; [ $rc -eq 0 ] || { tail -40 gpurun_out/segv_$TAG.err; exit $rc; }
  line gpurun_out/segv_$TAG.json segv
fi
if has c4sp; then   # c4 from span shards at N=1 (K1 build inside the step)
  timeout -k 10 600 python3 bench.py --config c4 --from-spans --steps 3 --warmup 1 --no-traffic --no-cpu > gpurun_out/c4sp_$TAG.json 2> gpurun_out/c4sp_$TAG.err || { tail -5 gpurun_out/c4sp_$TAG.err; exit 1; }
  line gpurun_out/c4sp_$TAG.json c4sp; python3 -c "import json;d=json.load(open('gpurun_out/c4sp_$TAG.json'));print('c4sp build_ms', d.get('build_ms'), 'ms_per_step', d['ms_per_step'])"
fi
if has c5s; then
  timeout -k 10 600 python3 bench.py --config c5 --from-spans --shard-of 8 --steps 3 --warmup 1 --no-traffic --no-cpu > gpurun_out/c5s_$TAG.json 2> gpurun_out/c5s_$TAG.err || { tail -5 gpurun_out/c5s_$TAG.err; exit 1; }
  line gpurun_out/c5s_$TAG.json c5s; python3 -c "import json;d=json.load(open('gpurun_out/c5s_$TAG.json'));print('c5s build_ms', d.get('build_ms'), 'ms_per_step', d['ms_per_step'])"
fi
if has pc5s; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pc5s_$TAG -o run --output-format csv \
      -- python3 bench.py --config c5 --from-spans --shard-of 8 --steps 2 --warmup 1 --no-traffic --no-cpu > gpurun_out/pc5s_$TAG.json 2> gpurun_out/pc5s_$TAG.err || { echo "rocprof pc5s failed"; tail -5 gpurun_out/pc5s_$TAG.err; exit 1; }
  line gpurun_out/pc5s_$TAG.json pc5s
fi
if has pc5; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pc5_$TAG -o run --output-format csv \
      -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-traffic --no-cpu > gpurun_out/pc5_$TAG.json 2> gpurun_out/pc5_$TAG.err || { echo "rocprof pc5 failed"; tail -5 gpurun_out/pc5_$TAG.err; exit 1; }
  line gpurun_out/pc5_$TAG.json pc5
fi
if has pc4s8; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pc4s8_$TAG -o run --output-format csv \
      -- python3 bench.py --config c4 --shard-of 8 --no-traffic --no-cpu --steps 5 --warmup 1 > gpurun_out/pc4s8_$TAG.json 2> gpurun_out/pc4s8_$TAG.err || { echo "rocprof pc4s8 failed"; tail -5 gpurun_out/pc4s8_$TAG.err; exit 1; }
  line gpurun_out/pc4s8_$TAG.json pc4s8
fi
# A/B of one environment knob on the c3 / c2 lines: AB_VAR, AB_VALS (space-separated), interleaved twice
if has c3ab || has c2ab; then
  for cfg in c3 c2; do
    has ${cfg}ab || continue
    for rep in 1 2; do
      for v in $AB_VALS; do
        vn=$(basename "$v")   # (a library path as the value: MR_LIB_PATH)
        env $AB_VAR=$v timeout -k 10 400 python3 bench.py --config $cfg --no-traffic --no-cpu --no-c4-leg > gpurun_out/ab_${cfg}_${TAG}_${vn}_$rep.json 2> gpurun_out/ab_${cfg}_${TAG}_${vn}_$rep.err || { tail -5 gpurun_out/ab_${cfg}_${TAG}_${vn}_$rep.err; exit 1; }
        line gpurun_out/ab_${cfg}_${TAG}_${vn}_$rep.json "$cfg $AB_VAR=$vn rep $rep"
      done
    done
  done
fi
# A/B of AB_VAR over AB_VALS on c4 (full) and c4 rank 0's share of 8, interleaved twice
if has c4ab; then
  for rep in 1 2; do
    for v in $AB_VALS; do
      for sh in 8 1; do
        env $AB_VAR=$v timeout -k 10 300 python3 bench.py --config c4 --shard-of $sh --steps 10 --warmup 2 --no-cpu --no-traffic > gpurun_out/ab_c4s${sh}_${TAG}_${v}_$rep.json 2> gpurun_out/ab_c4s${sh}_${TAG}_${v}_$rep.err || { tail -5 gpurun_out/ab_c4s${sh}_${TAG}_${v}_$rep.err; exit 1; }
        line gpurun_out/ab_c4s${sh}_${TAG}_${v}_$rep.json "c4 shard-of $sh $AB_VAR=$v rep $rep"
      done
    done
  done
fi
# A/B of AB_VAR over AB_VALS on the span-built c4 (N=1) and c5 (rank 0 of 8) steps, interleaved twice
if has spab; then
  for rep in 1 2; do
    for v in $AB_VALS; do
      env $AB_VAR=$v timeout -k 10 300 python3 bench.py --config c4 --from-spans --steps 3 --warmup 1 --no-traffic --no-cpu > gpurun_out/ab_c4sp_${TAG}_${v}_$rep.json 2> gpurun_out/ab_c4sp_${TAG}_${v}_$rep.err || { tail -5 gpurun_out/ab_c4sp_${TAG}_${v}_$rep.err; exit 1; }
      env $AB_VAR=$v timeout -k 10 300 python3 bench.py --config c5 --from-spans --shard-of 8 --steps 3 --warmup 1 --no-traffic --no-cpu > gpurun_out/ab_c5s_${TAG}_${v}_$rep.json 2> gpurun_out/ab_c5s_${TAG}_${v}_$rep.err || { tail -5 gpurun_out/ab_c5s_${TAG}_${v}_$rep.err; exit 1; }
      for c in c4sp c5s; do python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], 'build_ms', d.get('build_ms'), 'ms_per_step', d['ms_per_step'])" gpurun_out/ab_${c}_${TAG}_${v}_$rep.json "$c $AB_VAR=$v rep $rep"; done
    done
  done
fi
if has c3; then
  timeout -k 10 400 python3 bench.py --config c3 > gpurun_out/c3_$TAG.json 2> gpurun_out/c3_$TAG.err || { tail -5 gpurun_out/c3_$TAG.err; exit 1; }
  line gpurun_out/c3_$TAG.json c3
fi
if has c5; then
  timeout -k 10 600 python3 bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/c5_$TAG.json 2> gpurun_out/c5_$TAG.err || { tail -5 gpurun_out/c5_$TAG.err; exit 1; }
  line gpurun_out/c5_$TAG.json c5
fi
exit 0
