#!/bin/bash
# LDS anneal kernel (config B): per-run Verlet skin sweep (IGM_SKIN_SEG), full protocol,
# one warmup + one timed A/M iteration per variant -- tuning only.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/skinb
i=0
while IFS= read -r v; do
  i=$((i+1))
  if [ "$v" = "base" ]; then unset IGM_SKIN_SEG; else export IGM_SKIN_SEG="$v"; fi
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-de --no-c ${BARGS:-} \
    > gpurun_out/skinb/v$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; exit $rc; }
  python3 -c "
import json
for l in open('gpurun_out/skinb/v$i.log'):
    if l.startswith('{'):
        d=json.loads(l); b=d['breakdown']; print('skin=%-40s anneal_ms=%.1f step_ms=%.1f rebuilds=%.0f E/bead=%.3g' % ('$v', b['anneal_ms'], d['ms_per_step'], b['mean_rebuilds'], b['median_final_energy_per_bead']))"
done <<< "${VARIANTS:-base
0.7,1.0,0.7,0.8,0.7,0.7,0.7,0.6
0.7,1.3,0.7,0.9,0.7,0.7,0.7,0.5
0.5,1.0,0.5,0.8,0.5,0.6,0.5,0.4
0.7,0.7,0.7,0.7,0.7,0.5,0.7,0.4
0.5,0.9,0.5,0.7,0.5,0.5,0.5,0.35}"
