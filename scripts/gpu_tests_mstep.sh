#!/bin/bash
# M-step GPU tests touched by the engine work (parity of both HBM-size engines).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tm
timeout -k 10 900 python -u -m pytest tests/test_mstep_paths_gpu.py tests/test_configC_gpu.py tests/test_configDE_gpu.py \
  -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tm/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tm/tests.log | tail -25; exit $rc
