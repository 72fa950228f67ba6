#!/bin/bash
# A/B (config C pop=1000 x0.05): slot-space bond remap in the permute (default lib) against
# HEAD's atom-space re-index, and the force kernel at 7 waves per SIMD.
cd "$GRAFT_REPO_ROOT" || exit 1
L=igm_amd/lib/ab
TAG=ab3c ARGS="--config C --nstruct 1000 --protocol-scale 0.05" VARIANTS="IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_head.so
IGM_HIP_LIB=$L/libigmhip_o7.so
IGM_POP_GROUPS=2
IGM_HIP_LIB=$L/libigmhip_head.so
IGM_HIP_LIB=$L/libigmhip_o7.so" bash scripts/gpu_variants.sh
