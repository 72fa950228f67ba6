#!/bin/bash
# List capacity and fill batch of the population engine at the new skins (config C pop=1000 x0.05).
cd "$GRAFT_REPO_ROOT" || exit 1
L=igm_amd/lib/ab
TAG=ab6c ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS="IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_cap64.so
IGM_HIP_LIB=$L/libigmhip_cap56.so
IGM_HIP_LIB=$L/libigmhip_fw2.so
IGM_HIP_LIB=$L/libigmhip_fw6.so
IGM_POP_GROUPS=1
IGM_POP_GROUPS=2" bash scripts/gpu_variants.sh
