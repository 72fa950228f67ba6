#!/bin/bash
# Tuning sweep over env settings, one bench run per entry (tuning only).
#   RUNS="C:IGM_SKIN_FACTOR=0.55 C:IGM_SKIN_FACTOR=0.7 B:IGM_PROF=1"  SCALE_C=0.1 SCALE_B=0.2
# an entry is CONFIG[:VAR=value,VAR=value][:LIB] (LIB: igm_amd/lib/ab/libigmhip_LIB.so)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/tune_*.log
i=0
for r in $RUNS; do
  IFS=: read -r cfg envs lib <<< "$r"
  tag=$(echo "$r" | tr ':@=,' '____')
  (
    for kv in ${envs//,/ }; do export "$kv"; done
    [ -n "$lib" ] && export IGM_HIP_LIB=$PWD/igm_amd/lib/ab/libigmhip_$lib.so
    if [ "$cfg" = C ]; then sc=${SCALE_C:-0.1}; ns=${NSTRUCT_C:-125}; else sc=${SCALE_B:-0.2}; ns=${NSTRUCT_B:-1000}; fi
    timeout -k 10 600 python -u bench.py --config $cfg --nstruct $ns --protocol-scale $sc --steps 1 --warmup ${WARMUP:-0} \
      --cpu-sample 0 --no-de --no-c > gpurun_out/tune_$(printf %02d $i)_$tag.log 2>&1
  )
  rc=$?; echo "$r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
python scripts/show_tune.py
