"""bench_issue.json entry from the SQ counter passes of scripts/gpu_r02.sh:
    python scripts/make_issue.py profiles/<tag> [config B]
VALU-issue fraction = SQ_INSTS_VALU * SQ_WAVES / (SIMDs * SQ_WAVE_CYCLES): each SIMD's
cycles spent issuing wave64 VALU instructions (4 cycles each) over the cycles its
resident waves live (SQ_WAVE_CYCLES counts quad-cycles per wave)."""
import json
import os
import sys

d = sys.argv[1]
config = sys.argv[2] if len(sys.argv) > 2 else 'B'
v = {}
for fn in sorted(os.listdir(d)):
    if fn.startswith('sq') and fn.endswith('.txt'):
        for line in open(os.path.join(d, fn)):
            parts = line.split()
            if len(parts) >= 3 and parts[-3].startswith('SQ_'):
                v.setdefault(parts[-3], float(parts[-1]))
simds = 256 * 4
frac = v['SQ_INSTS_VALU'] * v['SQ_WAVES'] / (simds * v['SQ_WAVE_CYCLES'])
ent = {'bound': 'valu-issue', 'kernel': 'anneal_kernel<1024,3>', 'frac': frac,
       'achieved': v['SQ_INSTS_VALU'] / simds * 4.0, 'peak': v['SQ_WAVE_CYCLES'] * 4.0 / v['SQ_WAVES'],
       'unit': 'VALU issue cycles per SIMD over the launch',
       'lds_bank_conflict_frac': v.get('SQ_LDS_BANK_CONFLICT', 0.0) / max(v.get('SQ_LDS_IDX_ACTIVE', 1.0), 1.0),
       'wait_frac': v.get('SQ_WAIT_ANY', 0.0) / max(v.get('SQ_WAVE_CYCLES', 1.0), 1.0),
       'source': '%s/sq*.txt (rocprofv3 --pmc passes of bench.py --protocol-scale 0.05)' % d}
path = 'bench_issue.json'
cur = json.load(open(path)) if os.path.exists(path) else {}
cur[config] = ent
json.dump(cur, open(path, 'w'), indent=1)
print(json.dumps(ent))
