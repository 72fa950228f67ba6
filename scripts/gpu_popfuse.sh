#!/bin/bash
# Fused population engine: the pop-engine GPU tests, then a config C A/B (tuning).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_configC_gpu.py tests/test_mstep_paths_gpu.py tests/test_restraints_gpu.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/popfuse_tests.log 2>&1
rc=$?; tail -4 gpurun_out/popfuse_tests.log; [ $rc -eq 0 ] || exit $rc
RUNS=${RUNS:-"C::old C C::unf C"} bash scripts/gpu_sweep.sh
