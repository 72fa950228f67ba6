# bond pruning policy A/B: never / always / only when the replaced lists served >= AGE steps, on the frustrated
# shard and config E (scripts/dev/ab_de.py) and on the satisfiable 125-structure shard (full protocol)
VARIANTS="IGM_POP_BOND_PRUNE=0;IGM_POP_PRUNE_AGE=0;IGM_POP_PRUNE_AGE=3;IGM_POP_PRUNE_AGE=6;IGM_POP_BOND_PRUNE=0;IGM_POP_PRUNE_AGE=0" \
  BLOCKS=frustrated,E timeout -k 10 800 python3 -u scripts/dev/ab_de.py > gpurun_out/r06_abage.jsonl 2> gpurun_out/r06_abage.err
rc=$?; cat gpurun_out/r06_abage.jsonl; [ $rc -eq 0 ] || exit $rc
TAG=r06_abage ARGS="--config C --nstruct 125" TLIM=200 VARIANTS=$'IGM_POP_BOND_PRUNE=0\nIGM_POP_PRUNE_AGE=0\nIGM_POP_PRUNE_AGE=3\nIGM_POP_PRUNE_AGE=6' bash scripts/gpu_variants.sh
