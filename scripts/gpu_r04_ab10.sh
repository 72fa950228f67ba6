#!/bin/bash
# A/B: Verlet-list capacity of the population engine (row flushing), protocol x0.05, pop = 1000.
cd "$GRAFT_REPO_ROOT" || exit 1
L=igm_amd/lib/ab
ARGS="--config C --nstruct 1000 --protocol-scale 0.05" TLIM=240 TAG=${TAG:-r04_ab10} VARIANTS="IGM_HIP_LIB=$L/libigmhip_base.so
IGM_HIP_LIB=$L/libigmhip_fl128r40.so
IGM_HIP_LIB=$L/libigmhip_fl256r40.so
IGM_HIP_LIB=$L/libigmhip_fl384r40.so
IGM_HIP_LIB=$L/libigmhip_base.so
IGM_HIP_LIB=$L/libigmhip_fl256r40.so" bash scripts/gpu_variants.sh
