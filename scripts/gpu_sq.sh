#!/bin/bash
# SQ PMC pass (8 SQ counters, one run) over a short config-B bench (tuning only).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
CNT=${CNT:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"}
rm -rf gpurun_out/sq
timeout -s KILL 300 rocprofv3 --pmc $CNT -d gpurun_out/sq -o sq -- python3 bench.py --protocol-scale ${SCALE:-0.05} --steps 1 --warmup 0 --cpu-sample 0 --no-de ${BARGS:-} > gpurun_out/sq.log 2>&1
rc=$?; echo "sq rc=$rc"; exit $rc
