#!/bin/bash
# GPU suite, then the config B and C benches at the defaults (timing check).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/check
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/check/tests.log 2>&1
rc=$?; tail -3 gpurun_out/check/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-de --no-c > gpurun_out/check/b.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config C --steps 1 --warmup 1 --cpu-sample 0 --no-de > gpurun_out/check/c.log 2>&1 || exit $?
python3 -c "
import json
for f in ('b', 'c'):
    for l in open('gpurun_out/check/%s.log' % f):
        if l.startswith('{'):
            d=json.loads(l); b=d['breakdown']; print(f, 'anneal_ms=%.1f step_ms=%.1f rebuilds=%.0f value=%.3f' % (b['anneal_ms'], d['ms_per_step'], b['mean_rebuilds'], d['value']))"
