#!/bin/bash
# rocprofv3 kernel trace of the config C probe (population engine)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof -o kt -- python3 bench.py --config C --protocol-scale ${SCALE:-0.003} --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/cprof.log 2>&1
rc=$?; echo "cprof rc=$rc"; exit $rc
