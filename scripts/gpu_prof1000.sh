#!/bin/bash
# The metric's workload (config C, pop=1000) at a scaled protocol: kernel trace + HBM
# PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs).  usage: TAG=<dir> SCALE=<s> bash scripts/gpu_prof1000.sh
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r04_c1000}
SCALE=${SCALE:-0.05}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--config C --nstruct ${NSTRUCT:-1000} --protocol-scale $SCALE --steps 1 --warmup ${WARM:-1} --cpu-sample 0 --no-de $BARGS"
timeout -k 10 400 python -u bench.py $ARGS > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" $OUT/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py $ARGS > $OUT/prof_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -z "$NOPMC" ]; then
for CNT in FETCH_SIZE WRITE_SIZE; do
  D=$(echo $CNT | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 400 rocprofv3 --pmc $CNT -d $OUT/$D -o p -- python3 bench.py $ARGS > $OUT/p_$CNT.log 2>&1
  rc=$?; echo "pmc $CNT rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
fi
python3 scripts/prof_summary.py $OUT $OUT/sum > /dev/null; rm -rf $OUT/kt $OUT/fetch $OUT/write; head -12 $OUT/sum/kernel_stats.txt | cut -c1-160
