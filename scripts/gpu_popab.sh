#!/bin/bash
# population engine: HBM-path tests, then config C timings per variant (env settings)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mstep_paths_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pop_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pop_tests.log; [ $rc -eq 0 ] || exit $rc
SCALE=${SCALE:-0.05}
for V in ${VARIANTS:-"IGM_POP_GROUPS=1" "IGM_POP_GROUPS=4"}; do
  env $V timeout -k 10 600 python -u bench.py --config C --protocol-scale $SCALE --steps 1 --warmup 0 --cpu-sample 0 --no-de > gpurun_out/ab.log 2>&1
  rc=$?; echo "$V rc=$rc $(grep -o '"anneal_ms": [0-9.]*' gpurun_out/ab.log) $(grep -o '"mean_rebuilds": [0-9.]*' gpurun_out/ab.log)"; [ $rc -eq 0 ] || exit $rc
done
