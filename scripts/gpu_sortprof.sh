#!/bin/bash
# in-kernel phase stamps of pop_sort_kernel (variant libigmhip_sortprof.so; structure 0,
# every 200th rebuild) on config C, then a kernel-trace A/B of the variants
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
IGM_POP_GROUPS=1 IGM_HIP_LIB=$PWD/igm_amd/lib/ab/libigmhip_sortprof.so timeout -k 10 300 python -u bench.py --config C \
  --protocol-scale 0.2 --steps 1 --warmup 0 --cpu-sample 0 --no-de > gpurun_out/sortprof.log 2>&1
rc=$?; grep SORTPROF gpurun_out/sortprof.log | head -20; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profab.sh
