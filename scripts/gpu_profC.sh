#!/bin/bash
# Config C (200 kb) kernel trace on a scaled protocol: per-kernel time split of the
# population engine.  usage: TAG=<dir> SCALE=<protocol scale> bash scripts/gpu_profC.sh
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r02_c}
SCALE=${SCALE:-0.02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config C --protocol-scale $SCALE --steps 1 --warmup 0 --cpu-sample 0 --no-de \
    $BARGS > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" $OUT/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py --config C \
    --protocol-scale $SCALE --steps 1 --warmup 0 --cpu-sample 0 --no-de $BARGS > $OUT/prof_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $OUT $OUT/sum > /dev/null && rm -rf $OUT/kt && head -12 $OUT/sum/kernel_stats.txt | cut -c1-140
