"""Summarise rocprofv3 outputs (rocpd sqlite .db) of scripts/gpu_bench.sh into the
text files committed under profiles/<tag>/.

    python scripts/prof_summary.py gpurun_out/<tag> profiles/<tag>

kernel_stats.txt   per kernel: calls, total/avg duration (--kernel-trace --stats run)
hbm_traffic.txt    per kernel: FETCH_SIZE / WRITE_SIZE (separate --pmc runs), in KB as
                   rocprofv3 reports them, and the HBM bytes per launch after the
                   gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE x 2)
"""
import glob
import os
import sqlite3
import sys


def short(name, n=90):
    name = name.split('(')[0] if not name.startswith('(') else name
    return name if len(name) <= n else name[:n - 3] + '...'


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = list(c.execute('select name, count(*), sum(duration), avg(duration), max(grid_x / workgroup_x), '
                          'max(workgroup_x), max(vgpr_count), max(lds_size) from kernels group by name '
                          'order by 3 desc'))
    total = sum(r[2] for r in rows) or 1
    lines = ['%-90s %6s %14s %14s %7s %8s %5s %5s %7s' % ('kernel', 'calls', 'total_ms', 'avg_ms', 'pct', 'grid',
                                                         'wg', 'vgpr', 'lds')]
    for n, k, tot, avg, g, wg, vg, lds in rows:
        lines.append('%-90s %6d %14.3f %14.3f %7.3f %8d %5d %5d %7d' % (short(n), k, tot * 1e-6, avg * 1e-6,
                                                                       100.0 * tot / total, g, wg, vg, lds))
    return lines


def busy_union(db, pattern='pop_'):
    """GPU-busy share of the kernels matching `pattern`: the union of their [start, end)
    intervals over the span from the first start to the last end, and the mean number
    of them running at once (sum of durations / union)."""
    c = sqlite3.connect(db)
    iv = sorted(c.execute('select start, end from kernels where name like ?', ('%' + pattern + '%',)))
    if not iv:
        return None
    union, cur_s, cur_e, tot = 0, iv[0][0], iv[0][1], 0
    for a, b in iv:
        tot += b - a
        if a > cur_e:
            union += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    union += cur_e - cur_s
    span = max(b for _, b in iv) - iv[0][0]
    return {'span_ms': span * 1e-6, 'busy_ms': union * 1e-6, 'busy_frac': union / span,
            'mean_concurrency': tot / union, 'launches': len(iv)}


def launches(db, pattern):
    """every launch of the kernels matching `pattern` in dispatch order: (start offset
    from the first, duration) in ms -- the per-launch durations the bench's HIP events
    are compared with (launch 1 of a bench run is the warmup)"""
    c = sqlite3.connect(db)
    rows = list(c.execute('select name, start, end from kernels where name like ? order by start',
                          ('%' + pattern + '%',)))
    if not rows:
        return []
    t0 = rows[0][1]
    return [(short(n, 40), (a - t0) * 1e-6, (b - a) * 1e-6) for n, a, b in rows]


def pmc(db):
    c = sqlite3.connect(db)
    q = ('select kernel_name, counter_name, count(*), sum(value), avg(end - start) from counters_collection '
         'group by kernel_name, counter_name')
    return list(c.execute(q))


def pmc_by_anneal(db):
    """{counter: [bytes of the pop_* / anneal_kernel dispatches of anneal 1, 2, ...]}: the
    dispatches in id order, a new anneal at each run of pop_load launches (the groups'
    loads) or at each anneal_kernel launch, so a warmup anneal and a timed one are
    reported apart (value in KB as rocprofv3 gives FETCH_SIZE / WRITE_SIZE)"""
    c = sqlite3.connect(db)
    rows = list(c.execute('select dispatch_id, kernel_name, counter_name, sum(value) from counters_collection '
                          'group by dispatch_id, kernel_name, counter_name order by dispatch_id'))
    out, k, prev_load, last_id = {}, -1, False, None
    for did, name, cn, v in rows:
        is_load = 'pop_load' in name
        if did != last_id:
            if (is_load and not prev_load) or 'anneal_kernel' in name:
                k += 1
            prev_load = is_load
            last_id = did
        if k >= 0 and ('pop_' in name or 'anneal_kernel' in name):
            lst = out.setdefault(cn, [])
            while len(lst) <= k:
                lst.append(0.0)
            lst[k] += v
    return out


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    for db in glob.glob(os.path.join(src, 'kt', '*.db')):
        with open(os.path.join(dst, 'kernel_stats.txt'), 'w') as f:
            f.write('# rocprofv3 --kernel-trace --stats, %s\n' % os.path.basename(db))
            f.write('\n'.join(kernel_stats(db)) + '\n')
            for pat in ('pop_', 'anneal_kernel'):
                u = busy_union(db, pat)
                if u:
                    f.write('# busy union of %s kernels: %s\n' % (pat, u))
        with open(os.path.join(dst, 'anneal_launches.txt'), 'w') as f:
            f.write('# per-launch durations, dispatch order (launch 1 = warmup of the bench run); %s\n'
                    % os.path.basename(db))
            for pat in ('anneal_kernel', 'cg_kernel', 'classify_kernel', 'actdist_kernel'):
                for n, st, d in launches(db, pat):
                    f.write('%-40s start %12.3f ms  duration %12.3f ms\n' % (n, st, d))
            # the population engine: one anneal = the pop_* dispatches between two pop_load launches
            c = sqlite3.connect(db)
            rows = list(c.execute("select name, start, end from kernels where name like '%pop_%' order by start"))
            spans, cur, last_load = [], None, None
            for n, a, b in rows:
                if 'pop_load' in n and (last_load is None or a - last_load > 1e6):  # the groups' loads: one anneal
                    if cur:
                        spans.append(cur)
                    cur = [a, b]
                elif cur:
                    cur[1] = max(cur[1], b)
                if 'pop_load' in n:
                    last_load = a
            if cur:
                spans.append(cur)
            for k, (a, b) in enumerate(spans):
                f.write('population engine anneal %-15d span %12.3f ms (first pop_load .. last pop_* end)\n'
                        % (k + 1, (b - a) * 1e-6))
    out = ['# PMC passes (one counter per rocprofv3 run). value_KB = rocprofv3 FETCH_SIZE/WRITE_SIZE summed over',
           '# the launches; hbm_bytes_per_launch = KB*1024/calls, FETCH_SIZE doubled (gfx950 correction).',
           '%-70s %-10s %6s %18s %22s %14s' % ('kernel', 'counter', 'calls', 'value_KB', 'hbm_bytes_per_launch',
                                               'avg_ns')]
    for sub in ('fetch', 'write'):
        for db in glob.glob(os.path.join(src, sub, '*.db')):
            for k, cn, n, v, dur in pmc(db):
                corr = 2.0 if cn == 'FETCH_SIZE' else 1.0
                out.append('%-70s %-10s %6d %18.1f %22.4g %14.0f' % (short(k, 70), cn, n, v, v * 1024 * corr / n,
                                                                       dur))
    with open(os.path.join(dst, 'hbm_traffic.txt'), 'w') as f:
        f.write('\n'.join(out) + '\n')
        per = {}
        for sub in ('fetch', 'write'):
            for db in glob.glob(os.path.join(src, sub, '*.db')):
                for cn, v in pmc_by_anneal(db).items():
                    per[cn] = v
        if per:
            f.write('# per anneal (pop_* or anneal_kernel dispatches between anneal starts), HBM bytes after the\n'
                    '# gfx950 correction (FETCH_SIZE x 2): anneal 1 is the warmup launch of the bench run\n')
            for cn, v in sorted(per.items()):
                corr = 2.0 if cn == 'FETCH_SIZE' else 1.0
                f.write('%-10s %s\n' % (cn, '  '.join('anneal %d: %.4g' % (k + 1, x * 1024 * corr)
                                                     for k, x in enumerate(v))))
    for fn in ('bench.log', 'host.txt'):
        p = os.path.join(src, fn)
        if os.path.exists(p):
            with open(p) as fi, open(os.path.join(dst, fn.replace('.log', '.jsonl')), 'w') as fo:
                fo.write(''.join(l for l in fi if l.startswith('{') or fn == 'host.txt'))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
