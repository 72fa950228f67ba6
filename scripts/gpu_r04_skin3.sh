#!/bin/bash
# Full-protocol A/B of the population engine's skin rule at list capacity 256 (config C, 250
# structures, 1 warmup + 1 timed A/M iteration per variant); IGM_POP_SKIN_SEG runs in protocol
# order: relax, T0 = 5000, relax, 500, relax, 50, relax, 1.
cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="--config C --nstruct ${NS:-250} --protocol-scale 1.0" TLIM=${TLIM:-300} TAG=${TAG:-r04_skin3} VARIANTS="IGM_POP_SKIN_SEG=0.475,1.4,0.475,1.15,0.475,0.9,0.475,0.475
IGM_POP_SKIN_SEG=0.475,1.7,0.475,1.4,0.475,1.1,0.475,0.475
IGM_POP_SKIN_SEG=0.475,2.0,0.475,1.65,0.475,1.3,0.475,0.475
IGM_POP_SKIN_SEG=0.475,1.4,0.475,1.15,0.475,0.9,0.475,0.6" bash scripts/gpu_variants.sh
