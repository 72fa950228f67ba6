#!/bin/bash
# population-engine development loop: its GPU tests with the new library, then a
# kernel-trace A/B of the variants (scripts/gpu_profab.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mstep_paths_gpu.py tests/test_configC_gpu.py tests/test_mstep_stats.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/popdev_tests.log 2>&1
rc=$?; tail -3 gpurun_out/popdev_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profab.sh
