# kernel trace of the config E M-step block (125 structures, full protocol; scripts/dev/ab_de.py)
OUT=gpurun_out/r06_E
mkdir -p $OUT
export TMPDIR=/tmp
trap 'rm -rf $OUT/kt' EXIT
VARIANTS="IGM_POP_X=0" BLOCKS=E timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 -u scripts/dev/ab_de.py > $OUT/prof_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
mkdir -p $OUT/sum
python3 scripts/prof_summary.py $OUT $OUT/sum > /dev/null
head -12 $OUT/sum/kernel_stats.txt | cut -c1-150
grep "anneal" $OUT/sum/anneal_launches.txt
