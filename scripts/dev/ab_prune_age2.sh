# bond pruning age threshold, second sweep (scripts/dev/ab_prune_age.sh)
VARIANTS="IGM_POP_PRUNE_AGE=6;IGM_POP_PRUNE_AGE=10;IGM_POP_PRUNE_AGE=16;IGM_POP_BOND_PRUNE=0" \
  BLOCKS=frustrated,E timeout -k 10 800 python3 -u scripts/dev/ab_de.py > gpurun_out/r06_abage2.jsonl 2> gpurun_out/r06_abage2.err
rc=$?; cat gpurun_out/r06_abage2.jsonl; [ $rc -eq 0 ] || exit $rc
TAG=r06_abage2 ARGS="--config C --nstruct 125" TLIM=200 VARIANTS=$'IGM_POP_PRUNE_AGE=6\nIGM_POP_PRUNE_AGE=10\nIGM_POP_PRUNE_AGE=16\nIGM_POP_BOND_PRUNE=0\nIGM_POP_PRUNE_AGE=6\nIGM_POP_PRUNE_AGE=10' bash scripts/gpu_variants.sh
