#!/bin/bash
# Full bench line + rocprofv3 kernel trace + PMC HBM-traffic passes (one pass per run).
# The profiled runs use the bench's own step/warmup counts, so the per-launch anneal
# durations in the trace line up with the bench's timed launches (warmup = launch 1).
# usage: bash scripts/gpu_bench.sh <tag>   -> gpurun_out/<tag>/...
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
(nproc; lscpu | grep -i "model name"; rocm-smi --showproductname 2>/dev/null | head -20) > $OUT/host.txt 2>&1
BARGS=${BARGS:-}
timeout -k 10 900 python -u bench.py $BARGS > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
PARGS="--steps 2 --warmup 1 --cpu-sample 0 --no-de $BARGS"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py $PARGS > $OUT/prof_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch -- python3 bench.py $PARGS > $OUT/prof_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write -- python3 bench.py $PARGS > $OUT/prof_write.log 2>&1
rc=$?; echo "write rc=$rc"; exit $rc
