#!/bin/bash
# Population engine: parity tests of the changed kernels, then a per-run skin sweep on
# config C (full protocol, one warmup + one timed A/M iteration) -- tuning only.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/skinseg
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_configC_gpu.py tests/test_mstep_paths_gpu.py tests/test_restraints_gpu.py tests/test_configDE_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/skinseg/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/skinseg/tests.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
while IFS= read -r v; do
  i=$((i+1))
  if [ "$v" = "base" ]; then unset IGM_POP_SKIN_SEG; else export IGM_POP_SKIN_SEG="$v"; fi
  timeout -k 10 300 python -u bench.py --config C --nstruct 125 --steps 1 --warmup 1 --cpu-sample 0 --no-de \
    ${BARGS:-} > gpurun_out/skinseg/v$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; exit $rc; }
  python3 -c "
import json
for l in open('gpurun_out/skinseg/v$i.log'):
    if l.startswith('{'):
        d=json.loads(l); b=d['breakdown']; print('skin=%-40s anneal_ms=%.1f step_ms=%.1f rebuilds=%.0f E/bead=%.3g' % ('$v', b['anneal_ms'], d['ms_per_step'], b['mean_rebuilds'], b['median_final_energy_per_bead']))"
done <<< "${VARIANTS:-base
0.7,1.0,0.7,0.8,0.7,0.7,0.7,0.6
0.7,1.3,0.7,0.9,0.7,0.7,0.7,0.5
0.5,1.0,0.5,0.8,0.5,0.6,0.5,0.4
0.7,0.7,0.7,0.7,0.7,0.5,0.7,0.4}"
