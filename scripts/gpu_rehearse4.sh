#!/bin/bash
# Rehearsal of the N=4 bench line on ONE GPU (never a measurement): four ranks on cuda:0
# over gloo (IGM_BENCH_BACKEND=gloo: host-staged collectives), protocol x0.02, config B
# per rank (weak) and the config C pop=1000 strong split (250 per rank).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rehearse4
IGM_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 1 --warmup 1 --protocol-scale 0.02 \
  > gpurun_out/rehearse4/n4.log 2>&1
rc=$?; echo "rc=$rc"; grep "^{" gpurun_out/rehearse4/n4.log | cut -c1-600; exit $rc
