#!/bin/bash
# Tuning sweep: bench.py $ARGS under each line of $VARIANTS (environment settings),
# printing the anneal time and rebuild count of each.  usage:
#   ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS=$'A=1\nA=2' bash scripts/gpu_variants.sh
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-var}
mkdir -p $OUT
i=0
while IFS= read -r envs; do
  [ -z "$envs" ] && continue
  i=$((i+1))
  env $envs timeout -k 10 ${TLIM:-300} python -u bench.py ${ARGS:---config C --protocol-scale 0.05} --steps 1 \
    --warmup ${WARM:-1} --cpu-sample 0 --no-de > $OUT/v$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$envs rc=$rc"; tail -3 $OUT/v$i.log; exit $rc; }
  grep "^{" $OUT/v$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); b=d['breakdown']; print('%-60s anneal_ms=%.1f cg_ms=%.1f rebuilds=%.1f score=%.3g' % ('$envs', b['anneal_ms'], b['cg_ms'], b['mean_rebuilds'], b['violation_score']))"
done <<< "$VARIANTS"
