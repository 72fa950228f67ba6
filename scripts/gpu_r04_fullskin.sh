#!/bin/bash
# Full-protocol A/B of the population engine's skin rule and the velocity/flags split
# (config C, 250 structures, 1 warmup + 1 timed A/M iteration per variant).
cd "$GRAFT_REPO_ROOT" || exit 1
L=igm_amd/lib/ab
ARGS="--config C --nstruct ${NS:-250} --protocol-scale 1.0" TLIM=${TLIM:-420} TAG=${TAG:-r04_fullskin} VARIANTS="IGM_HIP_LIB=$L/libigmhip_head.so
IGM_HIP_LIB=$L/libigmhip_head.so IGM_POP_SKIN_SEG=0.45,1.0,0.45,0.855,0.45,0.705,0.45,0.45
IGM_HIP_LIB=$L/libigmhip_f3v.so
IGM_HIP_LIB=$L/libigmhip_head.so IGM_POP_SKIN_SEG=0.475,1.2,0.475,1.0,0.475,0.8,0.475,0.475
IGM_HIP_LIB=$L/libigmhip_f3v.so IGM_POP_SKIN_SEG=0.45,1.0,0.45,0.855,0.45,0.705,0.45,0.45" bash scripts/gpu_variants.sh
