#!/bin/bash
# Round-5 GPU experiments.  scripts/r05.sh TAG STAGES   (GPU box)
#   libab  : bench c2 (128 distinct windows, calls of 256, isolated group roofline) for every
#            library in LIBS (space-separated .so paths; MR_LIB_PATH), interleaved twice
#   pmcc2  : SQ LDS / wait counters of the c2 group k_tr_a launches (one pass, k_tr_a only)
#   pmcc2x : the same pass for every library in LIBS
TAG=${1:-x}; STAGES=${2:-libab}
has() { [[ " $STAGES " == *" $1 "* ]]; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline',{});i=r.get('isolated',{});print(sys.argv[2], d['value'], d.get('windows_per_s'), r.get('avg_launch_us'), r.get('frac'), i.get('avg_launch_us'), i.get('frac'), d.get('window_ms'))" "$1" "$2"; }
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
if has libab; then
  for rep in 1 2; do
    for lib in $LIBS; do
      vn=$(basename "$lib" .so)
      MR_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --no-c4-leg --c2-distinct 128 --steps 5 --warmup 1 \
          > gpurun_out/lab_${TAG}_${vn}_$rep.json 2> gpurun_out/lab_${TAG}_${vn}_$rep.err || { tail -5 gpurun_out/lab_${TAG}_${vn}_$rep.err; exit 1; }
      line gpurun_out/lab_${TAG}_${vn}_$rep.json "$vn rep $rep"
    done
  done
fi
if has pmcc2 || has pmcc2x; then
  L=${LIBS:-microrank_amd/libmicrorank_hip.so}
  has pmcc2x || L=microrank_amd/libmicrorank_hip.so
  for lib in $L; do
    vn=$(basename "$lib" .so)
    MR_LIB_PATH=$PWD/$lib timeout -s KILL 240 rocprofv3 --pmc $SQ --kernel-include-regex k_tr_a -d gpurun_out/pmc_${TAG}_$vn -o run --output-format csv -- \
        python3 bench.py --no-traffic --no-cpu --no-side --c2-distinct 64 --steps 1 --warmup 0 > gpurun_out/pmc_${TAG}_$vn.log 2>&1 || { echo "pmc $vn failed"; tail -5 gpurun_out/pmc_${TAG}_$vn.log; exit 1; }
    echo "== $vn"; python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_$vn k_tr_a | tee gpurun_out/pmc_${TAG}_$vn.txt
  done
fi
# envab: bench c2 (as libab) for every environment setting in ENVS (';'-separated, each a list of
# VAR=VAL words; "-" = none), interleaved twice
if has envab; then
  IFS=';' read -ra EV <<< "$ENVS"
  for rep in 1 2; do
    i=0
    for e in "${EV[@]}"; do
      i=$((i+1)); [ "$e" = "-" ] && e=""
      env $e timeout -k 10 300 python3 bench.py --no-traffic --no-cpu --no-c4-leg --c2-distinct 128 --steps 5 --warmup 1 \
          > gpurun_out/eab_${TAG}_${i}_$rep.json 2> gpurun_out/eab_${TAG}_${i}_$rep.err || { tail -5 gpurun_out/eab_${TAG}_${i}_$rep.err; exit 1; }
      line gpurun_out/eab_${TAG}_${i}_$rep.json "[$e] rep $rep"
    done
  done
fi
# pmcenv: the k_tr_a SQ pass of pmcc2 for every environment setting in ENVS
if has pmcenv; then
  IFS=';' read -ra EV <<< "$ENVS"
  i=0
  for e in "${EV[@]}"; do
    i=$((i+1)); [ "$e" = "-" ] && e=""
    env $e timeout -s KILL 240 rocprofv3 --pmc $SQ --kernel-include-regex k_tr_a -d gpurun_out/pmce_${TAG}_$i -o run --output-format csv -- \
        python3 bench.py --no-traffic --no-cpu --no-side --c2-distinct 64 --steps 1 --warmup 0 > gpurun_out/pmce_${TAG}_$i.log 2>&1 || { echo "pmc [$e] failed"; tail -5 gpurun_out/pmce_${TAG}_$i.log; exit 1; }
    echo "== [$e]"; python3 scripts/pmc_summary.py gpurun_out/pmce_${TAG}_$i k_tr_a | tee gpurun_out/pmce_${TAG}_$i.txt
  done
fi
# pmck: counter passes (PASSES: ';'-separated counter lists) over the kernels matching KRE in a
# short c2 bench, one rocprofv3 run per pass
if has pmck; then
  IFS=';' read -ra PS <<< "${PASSES:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS}"
  i=0
  for pc in "${PS[@]}"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $pc --kernel-include-regex "$KRE" -d gpurun_out/pmck_${TAG}_$i -o run --output-format csv -- \
        python3 bench.py --no-traffic --no-cpu --no-side --c2-distinct 64 --steps 1 --warmup 0 > gpurun_out/pmck_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmck_${TAG}_$i.log; exit 1; }
    echo "== pass $i"; python3 scripts/pmc_summary.py gpurun_out/pmck_${TAG}_$i "$KRE" | tee gpurun_out/pmck_${TAG}_$i.txt
  done
fi
