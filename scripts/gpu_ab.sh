#!/bin/bash
# A/B of libigmhip builds / tuning variables on the same box (tuning only).
#   VARIANTS="new old new" CONFIG=B SCALE=0.2 NSTRUCT=1000 SKIN=0.7
# a variant is LIB[@VAR=value,VAR=value]: LIB "new" = igm_amd/lib/libigmhip.so, any other
# name = igm_amd/lib/ab/libigmhip_LIB.so (scripts/build_variant.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/tune_*.log
i=0
for v in ${VARIANTS:-new old new}; do
  name=${v%%@*}; envs=""; [ "$name" != "$v" ] && envs=${v#*@}
  lib=igm_amd/lib/libigmhip.so; [ "$name" = new ] || lib=igm_amd/lib/ab/libigmhip_$name.so
  tag=$(echo "$v" | tr '@=,' '___')
  (
    for kv in ${envs//,/ }; do export "$kv"; done
    [ -n "$SKIN" ] && export IGM_SKIN_FACTOR=$SKIN
    IGM_HIP_LIB=$PWD/$lib timeout -k 10 600 python -u bench.py --config ${CONFIG:-B} --nstruct ${NSTRUCT:-1000} \
      --protocol-scale ${SCALE:-0.2} --steps 1 --warmup ${WARMUP:-0} --cpu-sample 0 --no-de --no-c > gpurun_out/tune_${CONFIG:-B}_${i}_$tag.log 2>&1
  )
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
python scripts/show_tune.py
