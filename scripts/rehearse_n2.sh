#!/bin/bash
# Rehearsal of the driver's N = 2 launch on a ONE-GPU box: both ranks on device 0 (MICRORANK_DEVICE),
# gloo control plane as in the driver's runs; the c4_sharded leg's RCCL cannot pair two ranks on
# one device, so that leg is expected to report an error while the line itself must complete.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MICRORANK_DEVICE=0 timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-traffic > gpurun_out/n2.json 2> gpurun_out/n2.err
rc=$?; echo "torchrun rc=$rc"
cut -c1-700 gpurun_out/n2.json
python3 -c "import json;d=json.load(open('gpurun_out/n2.json'));print('n_gpus',d['n_gpus'],'value',d['value'],'wps',d.get('windows_per_s'));print('c4', str(d.get('c4_sharded'))[:300]); print('cpu', d.get('cpu_baseline'))" || true
grep -i "error\|Traceback" gpurun_out/n2.err | head -10
exit $rc
