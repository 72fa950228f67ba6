#!/bin/bash
# Length-ranked force-kernel lanes: population-engine parity, then A/B against IGM_POP_BALANCE=0
# (config C pop=1000 x0.05), twice each.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bal
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_mstep_paths_gpu.py tests/test_configC_gpu.py tests/test_checkpoint_gpu.py -k "not full_protocol and not actdist" \
  > gpurun_out/bal/tests.log 2>&1
rc=$?; tail -4 gpurun_out/bal/tests.log; [ $rc -eq 0 ] || exit $rc
L=igm_amd/lib/ab
TAG=bal ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS="IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_bal0.so
IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_bal0.so" bash scripts/gpu_variants.sh
