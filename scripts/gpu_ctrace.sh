#!/bin/bash
# Kernel trace of the config C population engine (reduced protocol) for a timeline
# analysis of the per-step kernel chain -- tuning.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ctrace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ctrace/raw -o kt -- \
  python3 -u bench.py --config C --steps 1 --warmup 0 --cpu-sample 0 --no-de --protocol-scale ${PSCALE:-0.02} \
  > gpurun_out/ctrace/bench.log 2>&1 || exit $?
f=$(find gpurun_out/ctrace/raw -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" > gpurun_out/ctrace/timeline.txt 2>&1
rm -rf gpurun_out/ctrace/raw
tail -40 gpurun_out/ctrace/timeline.txt
