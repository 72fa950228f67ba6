#!/bin/bash
# pop-engine + contact-map GPU tests, then a config C A/B (tuning)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_configC_gpu.py tests/test_mstep_paths_gpu.py tests/test_restraints_gpu.py \
  tests/test_evaluation.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/popcsr_tests.log 2>&1
rc=$?; tail -4 gpurun_out/popcsr_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/gpu_contact.py > gpurun_out/contact_timing.log 2>&1; rc=$?; tail -5 gpurun_out/contact_timing.log; [ $rc -eq 0 ] || exit $rc
RUNS=${RUNS:-"C::old C C::old C"} bash scripts/gpu_sweep.sh
