#!/bin/bash
# GPU job: selected test files first (ARGS), then the whole -m gpu suite; fail fast.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FIRST=${FIRST:-}
if [ -n "$FIRST" ]; then
  timeout -k 10 700 python -u -m pytest $FIRST -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/first.log 2>&1
  rc=$?; tail -25 gpurun_out/first.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 1150 python -u -m pytest tests -m gpu -v -rfE --tb=long --timeout 800 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_all.log; exit $rc
