#!/bin/bash
# population-engine check: the HBM-path GPU tests, then the config C kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mstep_paths_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pop2_tests.log 2>&1
rc=$?; tail -15 gpurun_out/pop2_tests.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r02_c1} SCALE=${SCALE:-0.02} bash scripts/gpu_profC.sh
