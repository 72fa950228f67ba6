#!/bin/bash
# Counter calibration on the box (scripts/gather_calib.hip; build first: scripts/build_calib.sh):
# a plain run (unique bytes and HIP-event time per kernel), then one rocprofv3 --pmc pass per
# counter set, each summarised per kernel (summed over the REPS launches).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-calib}
mkdir -p $OUT
B=igm_amd/lib/calib/gather_calib
timeout -k 10 120 $B > $OUT/calib_times.json || exit 1
cat $OUT/calib_times.json
n=0
IFS=';' read -ra SS <<< "${SETS:-FETCH_SIZE;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum;TCC_EA0_RDREQ_DRAM_sum;WRITE_SIZE}"
for cs in "${SS[@]}"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $cs -d $OUT/p$n -o p -- $B > $OUT/p$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $n rc=$rc"; tail -3 $OUT/p$n.log; exit $rc; }
  python3 - $OUT/p$n <<'PY' | tee -a $OUT/calib_counters.txt
import glob, sqlite3, sys
db = glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
for kn, cn, k, v in c.execute('select kernel_name, counter_name, count(*), sum(value) from counters_collection '
                               'group by kernel_name, counter_name order by 1, 2'):
    print('%-20s %-24s %4d %.6g' % (kn.split('(')[0][-20:], cn, k, v))
PY
  rm -rf $OUT/p$n
done
exit 0
