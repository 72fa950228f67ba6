# bond batch width A/B on the 125-structure shard (full protocol)
TAG=r06_bb ARGS="--config C --nstruct 125" TLIM=200 VARIANTS=$'IGM_POP_X=0\nIGM_HIP_LIB=igm_amd/lib/ab/libigmhip_bb2.so\nIGM_HIP_LIB=igm_amd/lib/ab/libigmhip_bb1.so\nIGM_HIP_LIB=igm_amd/lib/ab/libigmhip_bb3.so\nIGM_POP_X=0\nIGM_HIP_LIB=igm_amd/lib/ab/libigmhip_bb2.so' bash scripts/gpu_variants.sh
