#!/bin/bash
# config C (200 kb) on a reduced protocol (timing probe)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --config C --nstruct ${NSTRUCT:-125} --sigma ${SIGMA:-0.01} --protocol-scale ${SCALE:-0.01} --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/tune_C.log 2>&1
rc=$?; echo "C rc=$rc"; exit $rc
