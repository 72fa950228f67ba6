#!/bin/bash
# A/B: brick slot order of the population engine (config C pop=1000 x0.05), twice each.
cd "$GRAFT_REPO_ROOT" || exit 1
L=igm_amd/lib/ab
TAG=ab2c ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS="IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_br4.so
IGM_HIP_LIB=$L/libigmhip_br2.so
IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_br4.so
IGM_HIP_LIB=$L/libigmhip_br2.so" bash scripts/gpu_variants.sh
