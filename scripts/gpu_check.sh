#!/bin/bash
# A GPU check in one call: selected tests (TESTS, pytest -k expression K), then optional
# anneal A/B variants (VARIANTS, scripts/gpu_variants.sh with ARGS) and an optional kernel
# trace (PROF=1: scripts/gpu_prof.sh with PARGS).  Every step under its own time limit;
# the first failing step ends the call.
#   TESTS="tests/test_mstep_paths_gpu.py" K="split_sort" VARIANTS=$'IGM_POP_SORT=1\nIGM_POP_SORT=0' \
#     ARGS="--config C --nstruct 125" bash scripts/gpu_check.sh
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-check}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTLIM:-600} python -u -m pytest $TESTS ${K:+-k "$K"} -x -v -rfE --tb=long --timeout 300 \
    --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$VARIANTS" ]; then
  TAG=${TAG:-check}/var bash scripts/gpu_variants.sh || exit 1
fi
if [ -n "$PROF" ]; then
  TAG=${TAG:-check}/prof PASSES=${PASSES:-kt} ARGS="$PARGS" bash scripts/gpu_prof.sh || exit 1
fi
exit 0
