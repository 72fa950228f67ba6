# skin rule re-check with bond pruning (125-structure shard, full protocol)
TAG=r06_skin ARGS="--config C --nstruct 125" TLIM=200 VARIANTS=$'IGM_POP_X=0\nIGM_POP_SKIN_RULE=0.4,0.25,1.3\nIGM_POP_SKIN_RULE=0.55,0.25,1.5\nIGM_POP_SKIN_RULE=0.475,0.2,1.3\nIGM_POP_X=0\nIGM_POP_SKIN_RULE=0.4,0.25,1.3' bash scripts/gpu_variants.sh
