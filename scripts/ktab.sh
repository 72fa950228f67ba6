#!/bin/bash
# One-group kernel traces (IGM_POP_GROUPS=1: no kernel overlap, so per-kernel durations add up) of
# bench.py $ARGS under each line of $VARIANTS (environment settings); prints the pop_* kernels'
# average durations and launch counts.  usage:
#   ARGS="--config C --nstruct 1000 --protocol-scale 0.02" VARIANTS=$'IGM_POP_WIN=0\nIGM_POP_WIN=1' bash scripts/ktab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp IGM_POP_GROUPS=1
OUT=gpurun_out/${TAG:-ktab}
mkdir -p $OUT
i=0
while IFS= read -r envs; do
  [ -z "$envs" ] && continue
  i=$((i+1))
  env $envs timeout -k 10 ${TLIM:-300} rocprofv3 --kernel-trace --stats -d $OUT/k$i -o kt -- python3 bench.py \
    ${ARGS:---config C --nstruct 1000 --protocol-scale 0.02} --steps 1 --warmup ${WARM:-1} --cpu-sample 0 --no-de \
    > $OUT/k$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$envs rc=$rc"; tail -3 $OUT/k$i.log; exit $rc; }
  python3 - $OUT/k$i "$envs" <<'PY'
import glob, sqlite3, sys
db = glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0]
rows = sqlite3.connect(db).execute('select name, count(*), sum(duration), avg(duration) from kernels group by name')
tot, out = 0.0, []
for n, k, s, a in rows:
    if 'pop_' in n:
        out.append('%s %.1f us x%d' % (n.split('pop_')[1].split('_kernel')[0], a / 1e3, k))
        tot += s
print('%-24s pop total %.0f ms | %s' % (sys.argv[2], tot / 1e6, ', '.join(sorted(out))))
PY
  [ -n "$KEEP" ] || rm -rf $OUT/k$i
done <<< "$VARIANTS"
