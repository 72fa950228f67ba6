"""Print the SQ counters of scripts/gpu_sq.sh per kernel: python scripts/sq_show.py [dir] [pattern]"""
import glob
import sqlite3
import sys

d = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/sq'
pat = sys.argv[2] if len(sys.argv) > 2 else 'anneal'
db = glob.glob(d + '/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute('select kernel_name, counter_name, count(*), sum(value) from counters_collection '
                 'group by kernel_name, counter_name')
for k, cn, n, v in rows:
    if pat in k:
        print('%-40s %-24s %4d %16.4g' % (k[:40], cn, n, v))
