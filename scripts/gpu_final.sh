#!/bin/bash
# Round-end rehearsal: the whole -m gpu suite, smoke(), config C bench; fail fast.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH_C" ]; then
  mkdir -p gpurun_out/benchC
  timeout -k 10 900 python -u bench.py --config C --steps 1 --warmup 0 --cpu-sample 0 --no-de > gpurun_out/benchC/bench.log 2>&1
  rc=$?; grep "^{" gpurun_out/benchC/bench.log | cut -c1-400; exit $rc
fi
