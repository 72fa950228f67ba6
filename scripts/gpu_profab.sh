#!/bin/bash
# kernel-trace A/B of libigmhip variants on config C (scaled protocol, one structure group)
#   VARIANTS="new old" SCALE=0.05 TAG=r02_kab
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r02_kab}; SCALE=${SCALE:-0.05}
export TMPDIR=/tmp IGM_POP_GROUPS=${IGM_POP_GROUPS:-1}
for v in ${VARIANTS:-new old}; do
  lib=igm_amd/lib/libigmhip.so; [ "$v" = new ] || lib=igm_amd/lib/ab/libigmhip_$v.so
  OUT=gpurun_out/$TAG/$v; mkdir -p $OUT
  IGM_HIP_LIB=$PWD/$lib timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py --config C \
      --protocol-scale $SCALE --steps 1 --warmup 0 --cpu-sample 0 --no-de > $OUT/prof_kt.log 2>&1
  rc=$?; echo "$v kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/prof_summary.py $OUT $OUT/sum > /dev/null && rm -rf $OUT/kt && echo "== $v" && head -9 $OUT/sum/kernel_stats.txt | cut -c1-130
done
