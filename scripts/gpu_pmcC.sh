#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a scaled config C run:
# HBM traffic, L2 hit rate and SQ issue counters of the population-engine kernels.
# usage: TAG=<dir> SCALE=<protocol scale> bash scripts/gpu_pmcC.sh
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r02_pmc}
SCALE=${SCALE:-0.05}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--config C --protocol-scale $SCALE --steps 1 --warmup 0 --cpu-sample 0 --no-de $BARGS"
i=0
while read -r CNT; do
  [ -z "$CNT" ] && continue
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $CNT -d $OUT/p$i -o p$i -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($CNT) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<L
${PASSES:-FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU}
L
python3 scripts/pmc_show.py $OUT pop_ > $OUT/pmc_pop.txt 2>&1
python3 scripts/pmc_show.py $OUT cg_kernel > $OUT/pmc_cg.txt 2>&1
rm -rf $OUT/p[0-9]*/
cat $OUT/pmc_pop.txt
