#!/bin/bash
# A/B: force-kernel bond hoist / occupancy (config C pop=1000 x0.05) and the anneal_kernel
# scratch fix (config B x0.2, against the HEAD build).
cd "$GRAFT_REPO_ROOT" || exit 1
L=igm_amd/lib/ab
TAG=ab1c ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS="IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_bf0.so
IGM_HIP_LIB=$L/libigmhip_bf5.so
IGM_HIP_LIB=$L/libigmhip_bf0o5.so" bash scripts/gpu_variants.sh || exit 1
TAG=ab1b ARGS="--protocol-scale 0.2 --no-c" VARIANTS="IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_head.so
IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_head.so" bash scripts/gpu_variants.sh
