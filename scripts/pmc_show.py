"""Per-kernel PMC table of scripts/gpu_pmcC.sh: python scripts/pmc_show.py gpurun_out/<tag> [pattern]
Values are summed over the launches and divided by the launch count (per launch)."""
import glob
import sqlite3
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else 'pop_'
acc = {}
for db in sorted(glob.glob(d + '/p*/**/*.db', recursive=True)):
    c = sqlite3.connect(db)
    q = 'select kernel_name, counter_name, count(distinct dispatch_id), sum(value) from counters_collection group by kernel_name, counter_name'
    try:
        rows = list(c.execute(q))
    except sqlite3.OperationalError:
        rows = list(c.execute('select kernel_name, counter_name, count(*), sum(value) from counters_collection '
                              'group by kernel_name, counter_name'))
    for k, cn, n, v in rows:
        if pat in k:
            acc.setdefault(k.split('(')[0][-40:], {})[cn] = (n, v / max(n, 1))
for k, cs in sorted(acc.items()):
    print(k)
    for cn, (n, v) in sorted(cs.items()):
        print('   %-24s %8d launches  %16.6g per launch' % (cn, n, v))
