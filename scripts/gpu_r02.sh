#!/bin/bash
# Round-2 measurement: the default bench line (config B + config C block + CPU
# baselines), then SQ counter passes over the config-B anneal kernel (instruction
# mix and stall/activity), one rocprofv3 --pmc run per pass.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r02_configB}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
(nproc; lscpu | grep -i "model name"; rocm-smi --showproductname 2>/dev/null | head -20) > $OUT/host.txt 2>&1
if [ -z "$NOBENCH" ]; then
  time timeout -k 10 900 python -u bench.py $BARGS > $OUT/bench.log 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc"; grep "^{" $OUT/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
fi
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P3="SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_MFMA_F32 SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES"
i=0
for CNT in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CNT -d $OUT/sq$i -o sq -- python3 bench.py --protocol-scale ${SCALE:-0.05} \
      --steps 1 --warmup 0 --cpu-sample 0 --no-de --no-c > $OUT/sq$i.log 2>&1
  rc=$?; echo "sq$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/sq_show.py $OUT/sq$i anneal > $OUT/sq$i.txt && rm -rf $OUT/sq$i
done
cat $OUT/sq*.txt
