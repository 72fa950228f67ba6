#!/bin/bash
# The driver's bench command (python bench.py --gpus 1 --steps 20 --warmup 5), timed by the
# wall clock around it, output under gpurun_out/<tag>/.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r04_bench}
mkdir -p gpurun_out/$TAG
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -i "model name"; rocm-smi --showproductname 2>/dev/null | head -20) > gpurun_out/$TAG/host.txt 2>&1
t0=$(date +%s.%N)
timeout -k 10 ${TLIM:-900} python3 -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARM:-5} $BARGS > gpurun_out/$TAG/bench.jsonl 2> gpurun_out/$TAG/bench.err
rc=$?
t1=$(date +%s.%N)
echo "rc=$rc wall_s=$(python3 -c "print($t1 - $t0)")" | tee gpurun_out/$TAG/wall.txt
cut -c1-400 gpurun_out/$TAG/bench.jsonl
exit $rc
