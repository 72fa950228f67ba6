#!/bin/bash
# Full bench line + rocprofv3 kernel trace + PMC HBM-traffic passes (one pass per run),
# summarised on the box (the raw rocpd databases exceed what gpurun brings back).
# The profiled runs use the bench's own step/warmup counts, so the per-launch anneal
# durations in the trace line up with the bench's timed launches (warmup = launch 1).
# usage: [BARGS=...] [PARGS=...] bash scripts/gpu_bench.sh <tag>   -> gpurun_out/<tag>/{bench.log,sum/}
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
(nproc; lscpu | grep -i "model name"; rocm-smi --showproductname 2>/dev/null | head -20) > $OUT/host.txt 2>&1
(while sleep 50; do date >> $OUT/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
BARGS=${BARGS:-}
if [ -z "$NOBENCH" ]; then
  timeout -k 10 900 python -u bench.py $BARGS > $OUT/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; grep "^{" $OUT/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
fi
PARGS=${PARGS:-"--steps 2 --warmup 1 --cpu-sample 0 --no-de --no-c $BARGS"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py $PARGS > $OUT/prof_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch -- python3 bench.py $PARGS > $OUT/prof_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write -- python3 bench.py $PARGS > $OUT/prof_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $OUT $OUT/sum && rm -rf $OUT/kt $OUT/fetch $OUT/write && head -8 $OUT/sum/kernel_stats.txt | cut -c1-140
