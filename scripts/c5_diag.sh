#!/bin/bash
# GPU box: C5 kernel traces of the default library and (if built) the A/B library, one iteration's
# launches each -> gpurun_out/c5d_TAG_*.txt (VARIANTS="def ab ab2": libmicrorank_hip_<v>.so)
#   scripts/c5_diag.sh TAG [bench args...]
TAG=${1:-x}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-def ab}; do
  if [ $v != def ]; then L=$PWD/microrank_amd/libmicrorank_hip_$v.so; [ -f "$L" ] || break; export MR_LIB_PATH=$L; else unset MR_LIB_PATH; fi
  D=gpurun_out/c5d_${TAG}_$v
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv \
      -- python3 bench.py --config c5 --no-traffic --no-cpu --steps 2 --warmup 1 "$@" > $D.json 2> $D.err || { tail -5 $D.err; exit 1; }
  f=$(find $D -name '*kernel_trace.csv' | head -1)
  python3 scripts/ktrace_iter.py "$f" 8 12 > ${D}_iter.txt
  s=$(find $D -name '*kernel_stats.csv' | head -1)
  python3 scripts/kstats.py "$s" 14 > ${D}_stats.txt
  echo "== $v"; cut -c1-300 $D.json; cat ${D}_iter.txt; head -16 ${D}_stats.txt
  rm -f "$f"
done
unset MR_LIB_PATH
