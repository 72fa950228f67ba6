#!/bin/bash
# the whole -m gpu suite, then a config B anneal A/B (scripts/gpu_ab.sh) of the variants
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
CONFIG=B NSTRUCT=1000 SCALE=${SCALE:-0.2} VARIANTS="${VARIANTS:-new old new}" bash scripts/gpu_ab.sh
