#!/bin/bash
# A/B of two libigmhip builds on the same box (tuning only).
#   VARIANTS="new old new" CONFIG=B SCALE=0.2 NSTRUCT=1000 SKIN=0.7
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/tune_*.log
i=0
for v in ${VARIANTS:-new old new}; do
  lib=igm_amd/lib/libigmhip.so; [ "$v" = old ] && lib=igm_amd/lib/ab/libigmhip_old.so
  IGM_SKIN_FACTOR=${SKIN:-1.0} IGM_HIP_LIB=$PWD/$lib timeout -k 10 600 python -u bench.py --config ${CONFIG:-B} --nstruct ${NSTRUCT:-1000} --protocol-scale ${SCALE:-0.2} --steps 1 --warmup 0 --cpu-sample 0 --no-de > gpurun_out/tune_${CONFIG:-B}_${i}_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
python scripts/show_tune.py
