#!/bin/bash
# Population-engine Verlet skin per run (IGM_POP_SKIN_SEG, units of the largest radius, runs in
# protocol order: relax, T0=5000, relax, 500, relax, 50, relax, 1) at pop=1000, config C x0.05.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=skin2 ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS="IGM_POP_GROUPS=2
IGM_POP_SKIN_SEG=0.45,1.2,0.45,1.0,0.45,0.8,0.45,0.45
IGM_POP_SKIN_SEG=0.45,1.4,0.45,1.15,0.45,0.9,0.45,0.45
IGM_POP_SKIN_SEG=0.45,1.6,0.45,1.3,0.45,1.0,0.45,0.45
IGM_POP_SKIN_SEG=0.45,1.4,0.45,1.3,0.45,1.1,0.45,0.45
IGM_POP_SKIN_SEG=0.45,1.8,0.45,1.5,0.45,1.2,0.45,0.45" bash scripts/gpu_variants.sh
L=igm_amd/lib/ab
TAG=ab5c ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS="IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_head.so
IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_head.so" bash scripts/gpu_variants.sh
