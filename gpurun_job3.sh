#!/bin/bash
# Full bench line + rocprofv3 kernel trace + PMC traffic passes (separate runs)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
nproc > gpurun_out/nproc.txt; lscpu | grep -i "model name" >> gpurun_out/nproc.txt
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o fetch -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o write -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof_write.log 2>&1
rc=$?; echo "write rc=$rc"; exit $rc
