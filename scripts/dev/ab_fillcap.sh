# permute/fill over a grid capped at IGM_POP_FILL_CAP structure slots, blocks looping over the flagged
# structures (A/B of the idle-block cost against one block per (structure, slot block) of the group)
TAG=r06_fcap ARGS="--config C --nstruct 125" TLIM=200 VARIANTS=$'IGM_POP_X=0\nIGM_POP_FILL_CAP=16\nIGM_POP_FILL_CAP=32\nIGM_POP_X=0\nIGM_POP_FILL_CAP=16\nIGM_POP_FILL_CAP=8' bash scripts/gpu_variants.sh
