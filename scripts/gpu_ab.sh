#!/bin/bash
# A/B of two libigmhip builds on the same box (tuning only): full protocol, 1 warmup + 1 timed step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-new old new}; do
  lib=igm_amd/lib/libigmhip.so; [ "$v" = old ] && lib=igm_amd/lib/libigmhip_old.so
  IGM_HIP_LIB=$PWD/$lib timeout -k 10 600 python -u bench.py --nstruct 1000 --protocol-scale ${SCALE:-1.0} --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/tune_ab_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cp gpurun_out/tune_ab_$v.log gpurun_out/ab_$v_$(date +%s).txt
done
