#!/bin/bash
# Config C (200 kb, 125 structures, FULL demo protocol) bench line + rocprofv3 kernel
# trace + FETCH_SIZE / WRITE_SIZE PMC passes (one counter per run), summarised on the
# box (the raw databases are too large to bring back).
# usage: [PRE="pytest args"] bash scripts/gpu_benchC.sh <tag>   -> gpurun_out/<tag>/sum/...
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02_configC}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$PRE" ]; then
  timeout -k 10 600 python -u -m pytest $PRE -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pre_tests.log 2>&1
  rc=$?; tail -3 $OUT/pre_tests.log; [ $rc -eq 0 ] || exit $rc
fi
(nproc; lscpu | grep -i "model name"; rocm-smi --showproductname 2>/dev/null | head -20) > $OUT/host.txt 2>&1
# a heartbeat under gpurun_out/ while the long, silent runs go (killed by its PID at exit)
(while sleep 50; do date >> $OUT/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
# (no CPU sample here: the config C CPU baseline is the scaled one of the default bench line)
timeout -k 10 900 python -u bench.py --config C --steps 1 --warmup 1 --cpu-sample 0 --no-de > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" $OUT/bench.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
PARGS="--config C --steps 1 --warmup 1 --cpu-sample 0 --no-de"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py $PARGS > $OUT/prof_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch -- python3 bench.py $PARGS > $OUT/prof_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write -- python3 bench.py $PARGS > $OUT/prof_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $OUT $OUT/sum && rm -rf $OUT/kt $OUT/fetch $OUT/write && head -12 $OUT/sum/kernel_stats.txt | cut -c1-140
