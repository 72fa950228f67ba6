#!/bin/bash
# Verlet skin per run at pop=1000 (config C x0.05): the default temperature rule against
# hotter/colder variants (IGM_SKIN_SEG, units of the largest radius, runs in protocol
# order: relax, T0=5000, relax, 500, relax, 50, relax, 1); and config B list/bond batch
# variants of the LDS kernel (x0.2).
cd "$GRAFT_REPO_ROOT" || exit 1
L=igm_amd/lib/ab
TAG=skin ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS="IGM_POP_GROUPS=2
IGM_SKIN_SEG=0.45,1.2,0.45,1.0,0.45,0.8,0.45,0.45
IGM_SKIN_SEG=0.45,0.85,0.45,0.73,0.45,0.6,0.45,0.45
IGM_SKIN_SEG=0.6,1.0,0.6,0.855,0.6,0.705,0.6,0.6
IGM_SKIN_SEG=0.4,1.0,0.4,0.855,0.4,0.705,0.4,0.4" bash scripts/gpu_variants.sh || exit 1
TAG=ab4b ARGS="--protocol-scale 0.2 --no-c" VARIANTS="IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_lpb4.so
IGM_HIP_LIB=$L/libigmhip_lpb1.so
IGM_HIP_LIB=$L/libigmhip_bb2.so
IGM_HIP_LIB=$L/libigmhip_lwb4.so
IGM_POP_GROUPS=2" bash scripts/gpu_variants.sh
