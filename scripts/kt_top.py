"""Top kernels of a rocprofv3 kernel-trace database: python scripts/kt_top.py <dir> [n]"""
import glob
import sqlite3
import sys

db = glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
for r in c.execute("select name, count(*), sum(duration)/1e6, avg(duration)/1e3 from kernels group by name "
                   "order by 3 desc limit %d" % (int(sys.argv[2]) if len(sys.argv) > 2 else 12)):
    print('%-60s %6d %10.2f ms %10.1f us' % (r[0][:60], r[1], r[2], r[3]))
