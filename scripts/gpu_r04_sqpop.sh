#!/bin/bash
# SQ counters of the population engine's kernels (config C, pop = 1000, protocol x0.02, one group):
# one rocprofv3 --pmc pass per counter set in $SETS (';'-separated), summed per kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp IGM_POP_GROUPS=1
OUT=gpurun_out/${TAG:-r04_sqpop}
mkdir -p $OUT
LIB=${LIB:-}
n=0
IFS=';' read -ra S <<< "${SETS:-SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE;TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE}"
for cs in "${S[@]}"; do
  n=$((n+1))
  IGM_HIP_LIB=${LIB:-igm_amd/lib/libigmhip.so} timeout -s KILL 300 rocprofv3 --pmc $cs -d $OUT/p$n -o p -- python3 bench.py --config C \
    --nstruct 1000 --protocol-scale 0.02 --steps 1 --warmup 1 --cpu-sample 0 --no-de > $OUT/p$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $n rc=$rc"; tail -3 $OUT/p$n.log; exit $rc; }
  python3 - $OUT/p$n <<'PY'
import glob, sqlite3, sys
db = glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
for kn, cn, k, v in c.execute('select kernel_name, counter_name, count(*), sum(value) from counters_collection '
                               'where kernel_name like "%pop_%" group by kernel_name, counter_name order by 1, 2'):
    print('%-14s %-24s %6d %.5g' % (kn.split('pop_')[1].split('_kernel')[0], cn, k, v))
PY
  rm -rf $OUT/p$n
done
