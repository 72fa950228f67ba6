"""bench_issue.json entry from the SQ pass of scripts/gpu_prof.sh (sum/sq_timed.txt, sq_last.py format):
    python scripts/make_issue.py profiles/<tag> [config B]
VALU-issue fraction of the SIMDs over the launch: a wave64 VALU instruction occupies
its SIMD-32 for 2 cycles (MI355X_MICROARCH.md "Wave scheduling"; 4 is the issue cost of
one wave alone, not the pipe occupancy), SQ_WAVE_CYCLES counts quad-cycles summed over
the waves (MI355X_MICROARCH.md cycle-constants table), so
    busy cycles per SIMD  = SQ_INSTS_VALU * 2 / SIMDs
    cycles per SIMD       = SQ_WAVE_CYCLES * 4 / SQ_WAVES   (every wave resident for the launch)
    frac                  = SQ_INSTS_VALU * SQ_WAVES / (2 * SIMDs * SQ_WAVE_CYCLES)."""
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
VALU_CYCLES = 2.0
frac = v['SQ_INSTS_VALU'] * VALU_CYCLES * v['SQ_WAVES'] / (simds * 4.0 * v['SQ_WAVE_CYCLES'])
ent = {'bound': 'latency' if v.get('SQ_WAIT_ANY', 0.0) / max(v.get('SQ_WAVE_CYCLES', 1.0), 1.0) > frac else 'valu-pipe', 'kernel': 'anneal_kernel<1024,3>', 'frac': frac,
       'achieved': v['SQ_INSTS_VALU'] / simds * VALU_CYCLES, 'peak': v['SQ_WAVE_CYCLES'] * 4.0 / v['SQ_WAVES'],
       'unit': 'VALU pipe cycles per SIMD over the launch (2 cycles per wave64 VALU instruction)',
       'lds_bank_conflict_frac': v.get('SQ_LDS_BANK_CONFLICT', 0.0) / max(v.get('SQ_LDS_IDX_ACTIVE', 1.0), 1.0),
       'wait_frac': v.get('SQ_WAIT_ANY', 0.0) / max(v.get('SQ_WAVE_CYCLES', 1.0), 1.0),
       'source': '%s/sq*.txt (%s)' % (d, sys.argv[3] if len(sys.argv) > 3 else 'rocprofv3 --pmc passes')}
path = 'bench_issue.json'
cur = json.load(open(path)) if os.path.exists(path) else {}
cur[config] = ent
json.dump(cur, open(path, 'w'), indent=1)
print(json.dumps(ent))
