#!/bin/bash
# GPU job: tests, smoke, short bench (each step time-limited; stop on any crash/timeout)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --nstruct 256 --protocol-scale 0.1 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench rc=$rc"
exit $rc
