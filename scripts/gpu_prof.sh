#!/bin/bash
# rocprofv3 passes over one bench.py regime, summarised on the box (the raw rocpd databases exceed
# what gpurun brings back).  PASSES: any of kt (kernel trace + stats), hbm (FETCH_SIZE and
# WRITE_SIZE, one counter per run), sq (one SQ pass; SQ_KERNEL names the kernel whose LAST
# dispatch -- the bench's timed launch -- is reported).  ARGS defaults to the metric's workload:
# config C, pop = 1000, full protocol, 1 warmup + 1 timed A/M iteration.
#   TAG=r05_C bash scripts/gpu_prof.sh
#   TAG=r05_B ARGS="--steps 1 --warmup 1 --cpu-sample 0 --no-de --no-c" SQ_KERNEL=anneal_kernel \
#     PASSES="kt hbm sq" bash scripts/gpu_prof.sh
# -> gpurun_out/<tag>/sum/{kernel_stats.txt, hbm_traffic.txt, sq_timed.txt}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-prof}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${ARGS:-"--config C --nstruct 1000 --steps 1 --warmup 1 --cpu-sample 0 --no-de"}
TLIM=${TLIM:-900}
SQ=${SQ:-"SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"}
(while sleep 50; do date >> $OUT/heartbeat.txt; done) &
HB=$!
# the raw rocpd databases exceed what gpurun brings back: removed on every exit, summarised first
trap 'kill $HB 2>/dev/null; rm -rf $OUT/kt $OUT/fetch $OUT/write $OUT/sqp' EXIT
for P in ${PASSES:-kt hbm}; do
  case $P in
    kt)
      timeout -k 10 $TLIM rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 -u bench.py $ARGS > $OUT/prof_kt.log 2>&1
      rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    hbm)
      for CNT in ${HBM_COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
        D=$(echo $CNT | cut -d_ -f1 | tr A-Z a-z)
        timeout -s KILL $TLIM rocprofv3 --pmc $CNT -d $OUT/$D -o p -- python3 -u bench.py $ARGS > $OUT/prof_$D.log 2>&1
        rc=$?; echo "pmc $CNT rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done ;;
    sq)
      timeout -s KILL $TLIM rocprofv3 --pmc $SQ -d $OUT/sqp -o sq -- python3 -u bench.py $ARGS > $OUT/prof_sq.log 2>&1
      rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
mkdir -p $OUT/sum
python3 scripts/prof_summary.py $OUT $OUT/sum > /dev/null
[ -d $OUT/sqp ] && python3 scripts/sq_last.py $OUT/sqp ${SQ_KERNEL:-pop_force} > $OUT/sum/sq_timed.txt
rm -rf $OUT/kt $OUT/fetch $OUT/write $OUT/sqp
ls $OUT/sum
head -8 $OUT/sum/kernel_stats.txt 2>/dev/null | cut -c1-150
tail -4 $OUT/sum/hbm_traffic.txt 2>/dev/null
cat $OUT/sum/sq_timed.txt 2>/dev/null
exit 0
