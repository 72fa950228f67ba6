#!/bin/bash
# Round-3 measurement job: the default bench line, the rocprofv3 kernel trace + PMC
# traffic passes of the config-B bench (scripts/gpu_bench.sh), then a kernel trace of
# the config-C bench summarised per protocol segment (scripts/stage_summary.py).
# usage: bash scripts/gpu_r03.sh <tag>   -> gpurun_out/<tag>/...
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/gpu_bench.sh $TAG || exit $?
if [ -z "$NOSTAGE" ]; then
  (while sleep 50; do date >> $OUT/heartbeat_c.txt; done) &
  HB=$!
  trap 'kill $HB 2>/dev/null' EXIT
  CARGS=${CARGS:-"--config C --steps 1 --warmup 1 --cpu-sample 0 --no-de"}
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/c/kt -o kt -- python3 bench.py $CARGS > $OUT/prof_ktc.log 2>&1
  rc=$?; echo "ktc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  mkdir -p $OUT/sumC
  python3 scripts/stage_summary.py $OUT/c > $OUT/sumC/stages.txt && python3 scripts/prof_summary.py $OUT/c $OUT/sumC && rm -rf $OUT/c
  grep "^{" $OUT/prof_ktc.log | cut -c1-400
  cat $OUT/sumC/stages.txt
fi
