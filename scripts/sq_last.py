"""SQ counters of the LAST dispatch of a kernel (the bench's timed launch, after the warmup
launch) from a rocprofv3 --pmc database, one line per counter (kernel, dispatch, counter, instances, value):
    python scripts/sq_last.py <dir> [kernel pattern] > profiles/<tag>/sq_timed.txt"""
import glob
import sqlite3
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else 'anneal_kernel'
for db in glob.glob(d + '/**/*.db', recursive=True):
    c = sqlite3.connect(db)
    last = c.execute('select max(dispatch_id) from counters_collection where kernel_name like ?',
                     ('%' + pat + '%',)).fetchone()[0]
    rows = c.execute('select kernel_name, counter_name, count(*), sum(value) from counters_collection '
                     'where dispatch_id = ? group by kernel_name, counter_name', (last,))
    for k, cn, n, v in rows:
        print('%-40s dispatch %-8d %-24s %4d %16.6g' % (k.split('(')[0][-40:], last, cn, n, v))
