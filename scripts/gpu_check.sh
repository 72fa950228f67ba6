#!/bin/bash
# GPU job: parity tests, smoke, short bench. Each step time-limited; stop at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --nstruct ${NSTRUCT:-256} --protocol-scale ${PSCALE:-0.1} --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
