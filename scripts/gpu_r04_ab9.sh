#!/bin/bash
# A/B: list-build batch (FILL_W) and quads collected in registers instead of an LDS row (REGQ); x0.05, pop = 1000.
cd "$GRAFT_REPO_ROOT" || exit 1
L=igm_amd/lib/ab
ARGS="--config C --nstruct 1000 --protocol-scale 0.05" TLIM=240 TAG=${TAG:-r04_ab9} VARIANTS="IGM_HIP_LIB=$L/libigmhip_t4.so
IGM_HIP_LIB=$L/libigmhip_w2.so
IGM_HIP_LIB=$L/libigmhip_rq24.so
IGM_HIP_LIB=$L/libigmhip_rq22.so
IGM_HIP_LIB=$L/libigmhip_rq44.so
IGM_HIP_LIB=$L/libigmhip_t4.so
IGM_HIP_LIB=$L/libigmhip_rq24.so
IGM_HIP_LIB=$L/libigmhip_pp.so
IGM_HIP_LIB=$L/libigmhip_pp.so" bash scripts/gpu_variants.sh
