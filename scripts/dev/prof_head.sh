# kernel traces at HEAD: config C pop = 1000 and the 125-structure shard (scripts/gpu_prof.sh, PASSES=kt)
TAG=r06_C_head PASSES=kt TLIM=600 bash scripts/gpu_prof.sh || exit 1
TAG=r06_s125_head PASSES=kt TLIM=300 ARGS="--config C --nstruct 125 --steps 1 --warmup 1 --cpu-sample 0 --no-de" bash scripts/gpu_prof.sh
