#!/bin/bash
# Full-protocol A/B of shorter hot-run skins at list capacity 256 (config C, 250 structures).
cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="--config C --nstruct ${NS:-250} --protocol-scale 1.0" TLIM=${TLIM:-300} TAG=${TAG:-r04_skin4} VARIANTS="IGM_POP_SKIN_SEG=0.475,1.4,0.475,1.15,0.475,0.9,0.475,0.475
IGM_POP_SKIN_SEG=0.475,1.2,0.475,1.0,0.475,0.8,0.475,0.475
IGM_POP_SKIN_SEG=0.475,1.0,0.475,0.855,0.475,0.705,0.475,0.475" bash scripts/gpu_variants.sh
