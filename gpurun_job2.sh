#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_mstep_gpu.py -q -p no:cacheprovider > gpurun_out/gpu_tests2.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --nstruct 256 --protocol-scale 0.1 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench rc=$rc"
exit $rc
