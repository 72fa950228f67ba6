#!/bin/bash
# Population-engine sweep (tuning only): structure groups x hardware queues on config C,
# protocol x SCALE, one warmup + one timed A/M iteration each; prints the anneal ms.
#   VARIANTS="2:4 4:4 4:8 ..."  (groups:queues)   SCALE=0.1
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/groups
for v in ${VARIANTS:-2:4 2:8 3:8 4:8 6:8 4:4}; do
  g=${v%%:*}; q=${v##*:}
  IGM_POP_GROUPS=$g GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --config C --nstruct 125 \
    --protocol-scale ${SCALE:-0.1} --steps 1 --warmup 1 --cpu-sample 0 --no-de > gpurun_out/groups/g${g}_q${q}.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "g=$g q=$q rc=$rc"; exit $rc; }
  python3 -c "
import json,sys
for l in open('gpurun_out/groups/g${g}_q${q}.log'):
    if l.startswith('{'):
        d=json.loads(l); b=d['breakdown']; print('groups=$g queues=$q anneal_ms=%.1f mstep_ms=%.1f step_ms=%.1f rebuilds=%.0f' % (b['anneal_ms'], b['mstep_ms'], d['ms_per_step'], b['mean_rebuilds']))"
done
