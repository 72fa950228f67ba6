#!/bin/bash
# A/B: list-build tail loads in flight (1 = serial, 4, 8); protocol x0.05, pop = 1000.
cd "$GRAFT_REPO_ROOT" || exit 1
L=igm_amd/lib/ab
ARGS="--config C --nstruct 1000 --protocol-scale 0.05" TLIM=240 TAG=${TAG:-r04_ab8} VARIANTS="IGM_HIP_LIB=$L/libigmhip_t1.so
IGM_HIP_LIB=$L/libigmhip_t4.so
IGM_HIP_LIB=$L/libigmhip_t8.so
IGM_HIP_LIB=$L/libigmhip_t1.so
IGM_HIP_LIB=$L/libigmhip_t4.so
IGM_HIP_LIB=$L/libigmhip_t8.so" bash scripts/gpu_variants.sh
