#!/bin/bash
# A/B of the default library vs microrank_amd/libmicrorank_hip_ab.so (MR_LIB_PATH), interleaved:
#   REPS=2 ARGS="--c2-distinct 64" scripts/gpu_ab.sh TAG      (GPU box; lines -> gpurun_out/ab_TAG_*.json)
#   AB_ENV="MR_X=0" ...: the "ab" runs take the default library with these variables set instead
#   VARIANTS="def ab ab2": libmicrorank_hip_<v>.so for each non-default variant
TAG=${1:-x}; REPS=${REPS:-2}; ARGS=${ARGS:-"--c2-distinct 64"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
AB=$PWD/microrank_amd/libmicrorank_hip_ab.so
for r in $(seq 1 $REPS); do
  for v in ${VARIANTS:-def ab}; do
    if [ $v != def ] && [ -z "$AB_ENV" ]; then export MR_LIB_PATH=$PWD/microrank_amd/libmicrorank_hip_$v.so; else unset MR_LIB_PATH; fi
    E=""; [ $v = ab ] && E="$AB_ENV"
    timeout -k 10 400 env $E python3 bench.py --no-traffic --no-cpu --no-side --steps 10 --warmup 2 $ARGS \
        > gpurun_out/ab_${TAG}_${v}_$r.json 2> gpurun_out/ab_${TAG}_${v}_$r.err || { tail -5 gpurun_out/ab_${TAG}_${v}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2], d['value'], d.get('windows_per_s'), r.get('avg_launch_us'), r.get('frac'), (r.get('u16_ids') or {}).get('frac'))" gpurun_out/ab_${TAG}_${v}_$r.json "$v$r"
  done
done
unset MR_LIB_PATH
