#!/bin/bash
# Population-engine parity after an engine change, then the config C pop=1000 x0.05 timing.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/check
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_configC_gpu.py tests/test_mstep_paths_gpu.py tests/test_configDE_gpu.py tests/test_checkpoint_gpu.py \
  > gpurun_out/check/tests.log 2>&1
rc=$?; tail -4 gpurun_out/check/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=check ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS="IGM_POP_GROUPS=2
IGM_POP_GROUPS=2" bash scripts/gpu_variants.sh
