"""Population-engine time per protocol segment (diagnostic, not product): from the
rocpd database of `rocprofv3 --kernel-trace` over bench.py --config C, the pop_*
kernel time of every anneal split at the segments' pop_setvel launches (one per
structure group and segment), per kernel.

    python scripts/stage_summary.py <dir with kt/*.db> > stages.txt
"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict

SEGS = ['relax1', 'stage1 5000->500', 'relax2', 'stage2 500->50', 'relax3', 'stage3 50->1', 'relax4',
        'stage4 1->0']


def main(src):
    db = glob.glob(os.path.join(src, 'kt', '*.db'))[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels where name like '%pop_%' order by start"))
    anneal, seg = -1, -1
    last_load = last_setvel = None
    acc = defaultdict(lambda: defaultdict(float))
    span = defaultdict(lambda: [None, None])
    cnt = defaultdict(int)
    for n, a, b in rows:
        if 'pop_load' in n:
            if last_load is None or a - last_load > 1e6:
                anneal += 1
                seg = -1
            last_load = a
            continue
        if 'pop_setvel' in n:
            if last_setvel is None or a - last_setvel > 1e5:
                seg += 1
            last_setvel = a
            continue
        key = (anneal, seg)
        k = n.split('(')[0].split('::')[-1].split('<')[0]
        acc[key][k] += (b - a) * 1e-6
        cnt[key] += 1
        sp = span[key]
        sp[0] = a if sp[0] is None else min(sp[0], a)
        sp[1] = b if sp[1] is None else max(sp[1], b)
    kinds = sorted({k for v in acc.values() for k in v})
    print('%-8s %-20s %10s %8s ' % ('anneal', 'segment', 'span_ms', 'launch') + ' '.join('%14s' % k for k in kinds))
    for key in sorted(acc):
        an, sg = key
        name = SEGS[sg] if 0 <= sg < len(SEGS) else str(sg)
        sp = span[key]
        print('%-8d %-20s %10.1f %8d ' % (an + 1, name, (sp[1] - sp[0]) * 1e-6, cnt[key]) +
              ' '.join('%14.1f' % acc[key].get(k, 0.0) for k in kinds))


if __name__ == '__main__':
    main(sys.argv[1])
