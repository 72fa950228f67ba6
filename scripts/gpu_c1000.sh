#!/bin/bash
# The metric's own workload on ONE GPU: 200 kb diploid, pop=1000, full demo protocol,
# 1 warmup + 1 timed A/M iteration (not part of the default bench line: ~5 minutes).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c1000
(while sleep 50; do date >> gpurun_out/c1000/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u bench.py --config C --nstruct 1000 --steps 1 --warmup 1 --cpu-sample 0 --no-de \
  > gpurun_out/c1000/bench.log 2>&1
rc=$?; grep "^{" gpurun_out/c1000/bench.log | cut -c1-400; exit $rc
