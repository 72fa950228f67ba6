#!/bin/bash
# Config B at HEAD, the bench's timed regime (1 warmup + 1 timed anneal, full protocol):
# kernel trace, FETCH_SIZE / WRITE_SIZE passes (one counter per run), one SQ pass; summaries
# written on the box under gpurun_out/<tag>/sum.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r04_B}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PARGS="--steps 1 --warmup 1 --cpu-sample 0 --no-de --no-c"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py $PARGS > $OUT/prof_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch -- python3 bench.py $PARGS > $OUT/prof_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write -- python3 bench.py $PARGS > $OUT/prof_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  -d $OUT/sqp -o sq -- python3 bench.py $PARGS > $OUT/prof_sq.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $OUT $OUT/sum > /dev/null && python3 scripts/sq_last.py $OUT/sqp > $OUT/sum/sq_timed.txt && \
  rm -rf $OUT/kt $OUT/fetch $OUT/write $OUT/sqp && head -6 $OUT/sum/kernel_stats.txt | cut -c1-150 && tail -4 $OUT/sum/hbm_traffic.txt && cat $OUT/sum/sq_timed.txt
