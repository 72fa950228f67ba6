#!/bin/bash
# Rehearsal of the N=8 bench line on ONE GPU (never a measurement): eight ranks on cuda:0 over
# gloo (IGM_BENCH_BACKEND=gloo: host-staged collectives), protocol x0.02, config B per rank
# (weak) and the config C pop=1000 strong split (the north-star shape: 125 structures per rank).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-rehearse8}
mkdir -p $OUT
IGM_BENCH_BACKEND=gloo timeout -k 10 ${TLIM:-900} python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --steps 1 --warmup 1 --protocol-scale 0.02 \
  --nstruct ${NSTRUCT:-250} > $OUT/n8.log 2>&1
rc=$?; echo "rc=$rc"; grep "^{" $OUT/n8.log > $OUT/n8.jsonl; cut -c1-400 $OUT/n8.jsonl; exit $rc
