#!/bin/bash
# profile the anneal with and without Hi-C bonds (tuning only)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for sg in ${SIGMAS:-1.1 0.02}; do
  IGM_PROF=1 timeout -k 10 600 python -u bench.py --nstruct 1000 --sigma $sg --protocol-scale ${SCALE:-1.0} --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/tune_sig$sg.log 2>&1
  rc=$?; echo "sigma $sg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
