#!/bin/bash
# Population engine: structure groups / chunking knobs on config C (protocol x0.1) -- tuning.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/grp
i=0
while IFS= read -r envs; do
  i=$((i+1))
  env $envs timeout -k 10 300 python -u bench.py --config C --steps 1 --warmup 1 --cpu-sample 0 --no-de \
    --protocol-scale ${PSCALE:-0.1} > gpurun_out/grp/v$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$envs rc=$rc"; tail -3 gpurun_out/grp/v$i.log; exit $rc; }
  grep "^{" gpurun_out/grp/v$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); b=d['breakdown']; print('%-40s anneal_ms=%.1f rebuilds=%.0f' % ('$envs', b['anneal_ms'], b['mean_rebuilds']))"
done <<< "${VARIANTS:-IGM_POP_GROUPS=2
IGM_POP_GROUPS=3
IGM_POP_GROUPS=1
IGM_POP_GROUPS=3}"
