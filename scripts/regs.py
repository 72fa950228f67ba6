"""Per-kernel register/spill summary of a HIP translation unit (development aid).
    python scripts/regs.py igm_amd/csrc/mstep.hip [extra hipcc flags]"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '--offload-arch=gfx950', '-fno-hip-fp32-correctly-rounded-divide-sqrt',
       '-munsafe-fp-atomics', '-Iinclude', '-c', src, '-o', '/tmp/_regs.o', '-Rpass-analysis=kernel-resource-usage'] + sys.argv[2:]
err = subprocess.run(cmd, stderr=subprocess.PIPE, text=True).stderr
cur = None
rows = {}
for line in err.splitlines():
    m = re.search(r'remark:\s+(.*?)\s*\[-Rpass', line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith('Function Name:'):
        cur = t.split(':', 1)[1].strip()
        rows[cur] = {}
    elif cur and ':' in t:
        k, v = t.split(':', 1)
        rows[cur][k.strip()] = v.strip()
names = subprocess.run(['c++filt'], input='\n'.join(rows), stdout=subprocess.PIPE, text=True).stdout.splitlines()
for (k, r), n in zip(rows.items(), names):
    if 'rocprim' in n:
        continue
    print('%-60s VGPR %4s spillV %4s spillS %4s scratch %5s occ %s' % (n.split('(')[0][:60], r.get('VGPRs'), r.get('VGPRs Spill'),
          r.get('SGPRs Spill'), r.get('ScratchSize [bytes/lane]'), r.get('Occupancy [waves/SIMD]')))
