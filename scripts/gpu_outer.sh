#!/bin/bash
# Population engine, two-level lists: parity tests with the outer list on, then config C
# (reduced protocol) per outer margin -- tuning.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/outer
if [ -z "$NOTEST" ]; then
  IGM_POP_OUTER=${TEST_OUTER:-0.5} timeout -k 10 600 python -u -m pytest tests/test_mstep_paths_gpu.py tests/test_configC_gpu.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/outer/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/outer/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for m in ${MARGINS:-0 0.3 0.5 0.8}; do
  IGM_POP_OUTER=$m timeout -k 10 300 python -u bench.py --config C --steps 1 --warmup 1 --cpu-sample 0 --no-de \
    --protocol-scale ${PSCALE:-0.1} > gpurun_out/outer/m$m.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "margin $m rc=$rc"; tail -5 gpurun_out/outer/m$m.log; exit $rc; }
  grep "^{" gpurun_out/outer/m$m.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); b=d['breakdown']; print('margin=%-4s anneal_ms=%.1f cg_ms=%.1f rebuilds=%.0f E/bead=%.3g viol=%.3g' % ('$m', b['anneal_ms'], b['cg_ms'], b['mean_rebuilds'], b['median_final_energy_per_bead'], b['violation_score']))"
done
