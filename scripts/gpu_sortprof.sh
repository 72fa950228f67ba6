#!/bin/bash
# Population engine sort kernel: phase profile at protocol x0.05 (needs a build with
# -DIGM_POP_SORT_PROF=1, scripts/build_variant.sh + IGM_HIP_LIB), then the config C anneal at
# x0.1 without profiling -- tuning.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sp
IGM_POP_SORT_PROF=1 timeout -k 10 300 python -u bench.py --config C --steps 1 --warmup 1 --cpu-sample 0 --no-de \
  --protocol-scale 0.05 > gpurun_out/sp/prof.log 2>&1 || exit $?
grep "pop sort" gpurun_out/sp/prof.log
timeout -k 10 300 python -u bench.py --config C --steps 1 --warmup 1 --cpu-sample 0 --no-de --protocol-scale 0.1 \
  > gpurun_out/sp/c.log 2>&1 || exit $?
grep "^{" gpurun_out/sp/c.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); b=d['breakdown']; print('x0.1 anneal_ms=%.1f rebuilds=%.0f E=%.3g' % (b['anneal_ms'], b['mean_rebuilds'], b['median_final_energy_per_bead']))"
