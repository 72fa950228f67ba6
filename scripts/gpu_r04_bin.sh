#!/bin/bash
# Binned rebuilds: the population-engine parity tests, then anneal time against the re-sort interval.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bin
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_configC_gpu.py -k "not full_protocol" \
  tests/test_mstep_paths_gpu.py tests/test_configDE_gpu.py > gpurun_out/bin/tests.log 2>&1
rc=$?; tail -15 gpurun_out/bin/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=bin ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS="IGM_POP_REORDER=1
IGM_POP_REORDER=4
IGM_POP_REORDER=8
IGM_POP_REORDER=16
IGM_POP_REORDER=64" bash scripts/gpu_variants.sh
