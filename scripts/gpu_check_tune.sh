#!/bin/bash
# M-step parity tests, then skin sweeps on B and C (tuning only).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mstep_gpu.py tests/test_mstep_paths_gpu.py tests/test_restraints_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ms_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ms_tests.log; [ $rc -eq 0 ] || exit $rc
FACTORS="${FB:-0.55 0.7 1.0}" CONFIG=B SCALE=0.2 PROF=1 bash scripts/gpu_skin.sh || exit 1
mkdir -p gpurun_out/tuneB && mv gpurun_out/tune_*.log gpurun_out/tuneB/
FACTORS="${FC:-0.55 0.7 1.0}" CONFIG=C NSTRUCT=125 SCALE=0.05 bash scripts/gpu_skin.sh || exit 1
