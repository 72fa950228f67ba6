#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config C --protocol-scale 0.01 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/tune_C.log 2>&1
rc=$?; echo "C rc=$rc"; [ $rc -eq 0 ] || exit $rc
IGM_FORCE_POP=1 timeout -k 10 600 python -u bench.py --nstruct 1000 --protocol-scale 0.1 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/tune_Bpop.log 2>&1
rc=$?; echo "Bpop rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --nstruct 1000 --protocol-scale 0.1 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/tune_Blds.log 2>&1
rc=$?; echo "Blds rc=$rc"; exit $rc
