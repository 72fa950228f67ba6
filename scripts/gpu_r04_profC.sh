#!/bin/bash
# The metric's workload (config C, pop=1000, FULL protocol, 1 warmup + 1 timed A/M iteration)
# under rocprofv3: PASS=kt (kernel trace) or PASS=pmc (FETCH_SIZE, WRITE_SIZE, one per run).
# Summaries on the box: gpurun_out/<tag>/sum (per-anneal split: anneal 2 is the timed one).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r04_C1000}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--config C --nstruct 1000 --steps 1 --warmup 1 --cpu-sample 0 --no-de"
if [ "${PASS:-kt}" = kt ]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 -u bench.py $ARGS > $OUT/prof_kt.log 2>&1
  rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
else
  for CNT in FETCH_SIZE WRITE_SIZE; do
    D=$(echo $CNT | cut -d_ -f1 | tr A-Z a-z)
    timeout -s KILL 540 rocprofv3 --pmc $CNT -d $OUT/$D -o p -- python3 -u bench.py $ARGS > $OUT/p_$CNT.log 2>&1
    rc=$?; echo "pmc $CNT rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
python3 scripts/prof_summary.py $OUT $OUT/sum_${PASS:-kt} > /dev/null; rm -rf $OUT/kt $OUT/fetch $OUT/write
ls $OUT/sum_${PASS:-kt}; head -8 $OUT/sum_${PASS:-kt}/kernel_stats.txt 2>/dev/null | cut -c1-150; tail -4 $OUT/sum_${PASS:-kt}/hbm_traffic.txt
