#!/bin/bash
# One-group kernel traces (IGM_POP_GROUPS=1: no kernel overlap) of config C, pop = 1000, protocol
# x${SCALE:-0.02}, for each library in $LIBS (names under igm_amd/lib/ab); prints the pop_* kernels' stats.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp IGM_POP_GROUPS=1
OUT=gpurun_out/${TAG:-r04_ktab}
mkdir -p $OUT
for v in $LIBS; do
  IGM_HIP_LIB=igm_amd/lib/ab/libigmhip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o kt -- python3 bench.py --config C --nstruct 1000 \
    --protocol-scale ${SCALE:-0.02} --steps 1 --warmup 1 --cpu-sample 0 --no-de > $OUT/$v.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 $OUT/$v.log; exit $rc; }
  python3 - $OUT/$v $v <<'PY'
import glob, sqlite3, sys
db = glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0]
rows = sqlite3.connect(db).execute('select name, count(*), sum(duration), avg(duration) from kernels group by name')
tot, out = 0.0, []
for n, k, s, a in rows:
    if 'pop_' in n:
        out.append('%s %.1f us x%d' % (n.split('pop_')[1].split('_kernel')[0], a / 1e3, k))
        tot += s
print(sys.argv[2], 'pop total %.0f ms |' % (tot / 1e6), ', '.join(sorted(out)))
PY
  rm -rf $OUT/$v
done
