#!/bin/bash
# A/B: velocity/flags split (f3v) against it with two list quads in flight (f3q2); protocol x0.05, pop = 1000.
cd "$GRAFT_REPO_ROOT" || exit 1
L=igm_amd/lib/ab
ARGS="--config C --nstruct 1000 --protocol-scale 0.05" TLIM=240 TAG=${TAG:-r04_ab7} VARIANTS="IGM_HIP_LIB=$L/libigmhip_f3v.so
IGM_HIP_LIB=$L/libigmhip_f3q2.so
IGM_HIP_LIB=$L/libigmhip_head.so
IGM_HIP_LIB=$L/libigmhip_f3v.so
IGM_HIP_LIB=$L/libigmhip_f3q2.so
IGM_HIP_LIB=$L/libigmhip_head.so" bash scripts/gpu_variants.sh
