#!/bin/bash
# Domain-decomposed engine bring-up: the direct checks, then the 200 kb parity tests,
# then config C at a reduced protocol on both engines (tuning).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dd
export IGM_DD_VERBOSE=1
timeout -k 10 240 python -u scripts/gpu_dd_check.py > gpurun_out/dd/check.log 2>&1
rc=$?; cat gpurun_out/dd/check.log | grep -v "^\[igm dd\]" | tail -20; [ $rc -eq 0 ] || exit $rc
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/dd/tests.log 2>&1
  rc=$?; tail -5 gpurun_out/dd/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for eng in ${ENGINES:-dd pop}; do
  IGM_POP_ENGINE=$eng timeout -k 10 300 python -u bench.py --config C --steps 1 --warmup 1 --cpu-sample 0 --no-de \
    --protocol-scale ${PSCALE:-0.1} > gpurun_out/dd/c_$eng.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $eng rc=$rc"; tail -5 gpurun_out/dd/c_$eng.log; exit $rc; }
  python3 -c "
import json
for l in open('gpurun_out/dd/c_$eng.log'):
    if l.startswith('{'):
        d=json.loads(l); b=d.get('breakdown', d.get('config_C', {}).get('breakdown', {})); c=d.get('config_C', d)
        b=c['breakdown']; print('$eng', 'anneal_ms=%.1f step_ms=%.1f rebuilds=%.0f E/bead=%.3g value=%.3f' % (b['anneal_ms'], c['ms_per_step'], b['mean_rebuilds'], b['median_final_energy_per_bead'], c['value']))"
  grep "^\[igm dd\]" gpurun_out/dd/c_$eng.log | tail -2
done
