#!/bin/bash
# Domain-decomposed engine: resident-set demand per domain count K on config C (the
# bench's warmup + timed A/M iterations at a reduced protocol) -- tuning only.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ddk
export IGM_DD_VERBOSE=1
for k in ${KS:-12 16 24}; do
  IGM_DD_K=$k timeout -k 10 300 python -u bench.py --config C --steps 1 --warmup 1 --cpu-sample 0 --no-de \
    --protocol-scale ${PSCALE:-0.02} > gpurun_out/ddk/k$k.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "K=$k rc=$rc"; tail -5 gpurun_out/ddk/k$k.log; exit $rc; }
  echo "K=$k"; grep "^\[igm dd\]" gpurun_out/ddk/k$k.log
done
