#!/bin/bash
# Round-6 GPU step: the -m gpu suite (optional) and bench lines -> gpurun_out/r06<TAG>_*
#   scripts/gpu_r06.sh TAG "t c2 c2ns c3 c4 c4s8 prof"
TAG=${1:-x}
STAGES=${2:-"t c2"}
has() { [[ " $STAGES " == *" $1 "* ]]; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r06${TAG}
if has t; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > ${O}_tests.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 ${O}_tests.txt; [ $rc -eq 0 ] || exit $rc
fi
if has s; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.txt 2>&1 || { tail -5 ${O}_smoke.txt; exit 1; }
fi
if has c2; then
  timeout -k 10 900 python3 bench.py > ${O}_c2.json 2> ${O}_c2.err || { tail -5 ${O}_c2.err; exit 1; }
  cut -c1-600 ${O}_c2.json
fi
if has c2ns; then
  timeout -k 10 600 python3 bench.py --no-traffic --no-cpu --no-c4-leg > ${O}_c2ns.json 2> ${O}_c2ns.err || { tail -5 ${O}_c2ns.err; exit 1; }
  cut -c1-600 ${O}_c2ns.json
fi
if has prof; then
  bash scripts/prof_bench.sh r06${TAG}_c2s --no-cpu --no-side --steps 10 --warmup 2 > /dev/null || exit 1
fi
for c in c3 c4 c5; do
  if has $c; then
    timeout -k 10 600 python3 bench.py --config $c > ${O}_$c.json 2> ${O}_$c.err || { tail -5 ${O}_$c.err; exit 1; }
    cut -c1-500 ${O}_$c.json
  fi
done
if has dropin; then
  timeout -k 10 400 python3 bench.py --config dropin > ${O}_dropin.json 2> ${O}_dropin.err || { tail -5 ${O}_dropin.err; exit 1; }
  cut -c1-400 ${O}_dropin.json
fi
if has pmc; then
  bash scripts/pmc_c2.sh r06${TAG} k_tr_a > ${O}_pmc.txt 2>&1 || { tail -5 ${O}_pmc.txt; exit 1; }
fi
if has c4s8; then
  bash scripts/prof_bench.sh r06${TAG}_c4s8 --config c4 --no-cpu --shard-of 8 --steps 10 --warmup 2 > /dev/null || exit 1
fi
echo done
