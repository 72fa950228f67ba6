#!/bin/bash
# population-engine kernel change: its GPU tests with the new library, then config C A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mstep_paths_gpu.py tests/test_configC_gpu.py tests/test_mstep_stats.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/force_tests.log 2>&1
rc=$?; tail -5 gpurun_out/force_tests.log; [ $rc -eq 0 ] || exit $rc
CONFIG=C NSTRUCT=125 SCALE=${SCALE:-0.2} VARIANTS="${VARIANTS:-new old pb2 new}" bash scripts/gpu_ab.sh
