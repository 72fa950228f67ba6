#!/bin/bash
# Config C, FULL demo protocol (1 warmup + 1 timed A/M iteration), domain-decomposed
# engine vs the population engine -- engine choice.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ddfull
export IGM_DD_VERBOSE=1
for eng in ${ENGINES:-dd pop}; do
  IGM_POP_ENGINE=$eng timeout -k 10 400 python -u bench.py --config C --steps 1 --warmup 1 --cpu-sample 0 --no-de \
    > gpurun_out/ddfull/$eng.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$eng rc=$rc"; tail -5 gpurun_out/ddfull/$eng.log; exit $rc; }
  echo "== $eng"; grep "^\[igm dd" gpurun_out/ddfull/$eng.log | tail -2
  grep "^{" gpurun_out/ddfull/$eng.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); b=d['breakdown']; print('anneal_ms=%.1f cg_ms=%.1f step_ms=%.1f rebuilds=%.0f E/bead=%.3g viol=%.3g' % (b['anneal_ms'], b['cg_ms'], d['ms_per_step'], b['mean_rebuilds'], b['median_final_energy_per_bead'], b['violation_score']))"
done
