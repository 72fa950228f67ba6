#!/bin/bash
# Parity tests + M-step launch-configuration sweep (tuning only).
#   CFGS="768x4 512x6"  SCALE=0.1  PROF=1  NOTEST=1
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CFGS:-768x4 512x6 1024x3}; do
  IGM_PROF=$PROF IGM_MD_CFG=$cfg timeout -k 10 600 python -u bench.py --nstruct 1000 --protocol-scale ${SCALE:-0.1} --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/tune_$cfg.log 2>&1
  rc=$?; echo "cfg $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
