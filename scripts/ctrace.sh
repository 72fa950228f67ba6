#!/bin/bash
# Kernel-trace timelines (scripts/timeline.py: per-kernel durations, busy union, gaps) of the config C
# population engine at the default two structure groups, one per line of $VARIANTS (environment settings).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ctrace}
mkdir -p $OUT
i=0
while IFS= read -r envs; do
  [ -z "$envs" ] && continue
  i=$((i+1))
  env $envs timeout -k 10 ${TLIM:-300} rocprofv3 --kernel-trace --output-format csv -d $OUT/raw$i -o kt -- \
    python3 -u bench.py ${ARGS:---config C --nstruct 1000 --protocol-scale 0.02} --steps 1 --warmup 1 --cpu-sample 0 \
    --no-de > $OUT/b$i.log 2>&1 || { echo "$envs rc=$?"; exit 1; }
  f=$(find $OUT/raw$i -name "*kernel_trace.csv" | head -1)
  echo "== $envs" > $OUT/t$i.txt
  python3 scripts/timeline.py "$f" >> $OUT/t$i.txt 2>&1
  rm -rf $OUT/raw$i
  head -16 $OUT/t$i.txt
done <<< "$VARIANTS"
