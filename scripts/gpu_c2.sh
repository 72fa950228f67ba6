#!/bin/bash
# config C probes: with / without Hi-C bonds, kernel trace (tuning only)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for sg in ${SIGMAS:-1.1 0.01}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof_$sg -o kt -- python3 bench.py --config C --sigma $sg --protocol-scale ${SCALE:-0.003} --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/cprof_$sg.log 2>&1
  rc=$?; echo "sigma $sg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
