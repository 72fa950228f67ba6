#!/bin/bash
# anneal-kernel phase profile (cycle counters) on the reduced and full protocol
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ps in ${SCALES:-0.1 1.0}; do
  IGM_PROF=1 timeout -k 10 300 python -u bench.py --nstruct ${NSTRUCT:-1000} --protocol-scale $ps --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof_$ps.log 2>&1
  rc=$?; echo "scale $ps rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
