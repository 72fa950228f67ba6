#!/bin/bash
# Config B (2 Mb, 1000 structures, LDS engine), full protocol: the LDS engine's per-run skin rule
# against longer / shorter hot-run skins (IGM_SKIN_SEG, runs in protocol order: relax, T0 = 5000,
# relax, 500, relax, 50, relax, 1; units of the largest radius).
cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="--no-c --protocol-scale 1.0" TLIM=${TLIM:-200} TAG=${TAG:-r04_skinB} VARIANTS="IGM_SKIN_SEG=0.45,1.0,0.45,0.855,0.45,0.705,0.45,0.45
IGM_SKIN_SEG=0.45,1.2,0.45,1.0,0.45,0.8,0.45,0.45
IGM_SKIN_SEG=0.45,0.85,0.45,0.73,0.45,0.6,0.45,0.45
IGM_SKIN_SEG=0.45,1.0,0.45,0.855,0.45,0.705,0.45,0.45
IGM_SKIN_SEG=0.45,1.2,0.45,1.0,0.45,0.8,0.45,0.45
IGM_SKIN_SEG=0.5,1.0,0.5,0.855,0.5,0.705,0.5,0.5" bash scripts/gpu_variants.sh
