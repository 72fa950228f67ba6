#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter set in $SETS, ';'-separated) of bench.py $ARGS,
# summed per kernel whose name matches $MATCH (sqlite LIKE pattern).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
n=0
IFS=';' read -ra SS <<< "${SETS:-SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE}"
for cs in "${SS[@]}"; do
  n=$((n+1))
  timeout -s KILL 300 rocprofv3 --pmc $cs -d $OUT/p$n -o p -- python3 bench.py ${ARGS:---steps 1 --warmup 0 \
    --protocol-scale 0.02 --cpu-sample 0 --no-c} > $OUT/p$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $n rc=$rc"; tail -3 $OUT/p$n.log; exit $rc; }
  python3 - $OUT/p$n "${MATCH:-%}" <<'PY'
import glob, sqlite3, sys
db = glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
for kn, cn, k, v in c.execute('select kernel_name, counter_name, count(*), sum(value) from counters_collection '
                               'where kernel_name like ? group by kernel_name, counter_name order by 1, 2', (sys.argv[2],)):
    print('%-28s %-26s %6d %.5g' % (kn.split('(')[0][-28:], cn, k, v))
PY
  rm -rf $OUT/p$n
done
