"""Scratch (spill / private-array) instructions of one kernel by loop depth, from a
device assembly file (development aid):
    hipcc ... --cuda-device-only -S igm_amd/csrc/mstep.hip -o /tmp/mstep.s
    python scripts/scratch_depth.py /tmp/mstep.s anneal_kernelILi1024ELi3E"""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
start = [k for k, l in enumerate(lines) if re.match(r'^_Z\w*%s\w*:' % sys.argv[2], l)][0]
end = [k for k in range(start + 1, len(lines)) if lines[k].startswith('.Lfunc_end')][0]
depth, cnt = 0, {}
for l in lines[start:end]:
    if re.match(r'^\.LBB', l) or l.strip().startswith('; %bb'):
        m = re.search(r'Depth=(\d+)', l)
        depth = int(m.group(1)) if m else 0
    if 'scratch_' in l:
        op = l.split()[0]
        cnt[(depth, op)] = cnt.get((depth, op), 0) + 1
for k in sorted(cnt):
    print('depth %d  %-24s %d' % (k[0], k[1], cnt[k]))
