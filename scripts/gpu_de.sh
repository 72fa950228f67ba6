#!/bin/bash
# The D/E A-step kernels: their GPU tests, the bench's asteps_DE timing (200 kb x 1000
# structures), and a rocprofv3 kernel trace of the same block (per-kernel average durations).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-de}
mkdir -p $OUT
export TMPDIR=/tmp
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
[ -n "$NOKT" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py --steps 1 --warmup 0 \
  --protocol-scale 0.01 --cpu-sample 0 --no-c > $OUT/kt.log 2>&1 || exit $?
python3 - $OUT/kt > $OUT/kernels_de.txt <<'PY'
import glob, sqlite3, sys
db = glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0]
for n, k, s, a in sqlite3.connect(db).execute('select name, count(*), sum(duration), avg(duration) from kernels group by name order by 3 desc'):
    if any(x in n for x in ('sprite', 'fish', 'polymer', 'damid')):
        print('%-60s x%-4d avg %.1f us' % (n.split('(')[1] if n.startswith('(') else n[:60], k, a / 1e3))
PY
rm -rf $OUT/kt
cat $OUT/kernels_de.txt
