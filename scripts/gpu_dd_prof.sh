#!/bin/bash
# Domain-decomposed engine: per-phase wall-clock profile on config C (reduced protocol) -- tuning only.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ddp
export IGM_DD_VERBOSE=1 IGM_DD_PROF=1
i=0
while IFS= read -r envs; do
  i=$((i+1))
  env $envs timeout -k 10 300 python -u bench.py --config C --steps 1 --warmup 1 --cpu-sample 0 --no-de \
    --protocol-scale ${PSCALE:-0.02} > gpurun_out/ddp/v$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$envs rc=$rc"; tail -5 gpurun_out/ddp/v$i.log; exit $rc; }
  echo "== $envs"; grep "^\[igm dd" gpurun_out/ddp/v$i.log | tail -2
  grep "^{" gpurun_out/ddp/v$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); b=d['breakdown']; print('anneal_ms=%.1f cg_ms=%.1f rebuilds=%.0f E/bead=%.3g' % (b['anneal_ms'], b['cg_ms'], b['mean_rebuilds'], b['median_final_energy_per_bead']))"
done <<< "${VARIANTS:-IGM_DD_K=24
IGM_DD_K=24 IGM_DD_TOL=0.1}"
