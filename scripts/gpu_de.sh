#!/bin/bash
# The D/E A-step kernels: their GPU tests, then the bench's asteps_DE block (200 kb x 1000 structures).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-de}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_asteps_gpu.py \
  tests/test_polymer.py tests/test_steps_de.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --protocol-scale 0.02 --cpu-sample 0 --no-c > $OUT/b.jsonl \
  2>/dev/null || exit $?
python - $OUT/b.jsonl <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['asteps_DE']
for k in ('damid', 'fish', 'sprite', 'polymer'):
    print('%-8s %8.3f ms %6.0f GB/s' % (k, d[k]['ms'], d[k]['achieved_GBps']))
PY
