#!/bin/bash
# GPU job: configuration D/E A-step parity tests (time-limited).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_asteps_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/asteps_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/asteps_gpu.log; exit $rc
