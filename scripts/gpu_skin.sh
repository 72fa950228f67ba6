#!/bin/bash
# Verlet skin sweep (tuning only; LAMMPS semantics make the skin a performance knob).
#   FACTORS="0.5 0.7 1.0"  CONFIG=B  SCALE=0.2  NSTRUCT=1000
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/tune_*.log
for f in ${FACTORS:-0.5 0.7 1.0}; do
  IGM_PROF=$PROF IGM_SKIN_FACTOR=$f timeout -k 10 600 python -u bench.py --config ${CONFIG:-B} --nstruct ${NSTRUCT:-1000} --protocol-scale ${SCALE:-0.2} --steps 1 --warmup 0 --cpu-sample 0 --no-de > gpurun_out/tune_${CONFIG:-B}_skin$f.log 2>&1
  rc=$?; echo "skin $f rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/show_tune.py
