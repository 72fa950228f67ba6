"""Timeline of the population engine's per-step kernel chain from a rocprofv3 kernel
trace (csv): per kernel name the mean duration, the busy union of pop_* kernels, the
mean gap between a kernel's end and the next launch on the same stream, and a sample
window of consecutive launches."""
import csv
import sys
from collections import defaultdict

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        n = r['Kernel_Name']
        if 'pop_' not in n:
            continue
        short = n.split('(')[0].replace('void ', '').replace('igm::ms::', '')
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), short, r.get('Stream_Id', r.get('Queue_Id', '?'))))
rows.sort()
print('pop_* launches', len(rows))
t0, t1 = rows[0][0], rows[-1][1]
# busy union
busy, cur_s, cur_e = 0, None, None
for s, e, _, _ in rows:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print('span %.1f ms busy-union %.1f ms (%.1f%%)' % ((t1 - t0) / 1e6, busy / 1e6, 100.0 * busy / (t1 - t0)))
dur = defaultdict(list)
for s, e, n, q in rows:
    dur[n].append(e - s)
for n, v in sorted(dur.items(), key=lambda x: -sum(x[1])):
    v = sorted(v)
    print('%-40s n=%6d mean %7.1f us  p50 %7.1f  p90 %7.1f  total %8.1f ms' % (
        n[:40], len(v), sum(v) / len(v) / 1e3, v[len(v) // 2] / 1e3, v[int(len(v) * 0.9)] / 1e3, sum(v) / 1e6))
# gaps per stream: next start - previous end
bys = defaultdict(list)
for s, e, n, q in rows:
    bys[q].append((s, e, n))
for q, v in bys.items():
    gaps = [max(0, v[i + 1][0] - v[i][1]) for i in range(len(v) - 1)]
    if gaps:
        gs = sorted(gaps)
        print('stream %s: launches %d, gap mean %.1f us p50 %.1f p90 %.1f' % (q, len(v), sum(gs) / len(gs) / 1e3,
                                                                            gs[len(gs) // 2] / 1e3, gs[int(len(gs) * .9)] / 1e3))
# a sample window in the last third
mid = rows[int(len(rows) * 0.8)][0]
print('--- window')
for s, e, n, q in rows:
    if mid <= s < mid + 1200000:
        print('%9.1f %9.1f %7.1f  q%s %s' % ((s - mid) / 1e3, (e - mid) / 1e3, (e - s) / 1e3, q, n[:40]))
