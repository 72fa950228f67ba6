"""Time igm_contact_map (HicEvaluationStep contact map) on synthetic populations.
pair-structure checks/s and the VALU op rate (10 f32 ops per check: 3 sub, 3 mul,
2 add, compare, add) against the f32 vector peak."""
import json
import sys

import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from igm_amd import _lib, evaluation as EV

c = _lib.context(0)
res = []
for nbead, S in [(3008, 1000), (12000, 1000)]:
    rng = np.random.default_rng(1)
    xyz = (rng.standard_normal((nbead, S, 3)) * 1500).astype(np.float32)
    r = np.full(nbead, 118.0, np.float32)
    EV.contact_counts(xyz, r, 2.0, ctx=c)  # warm
    ms = []
    for _ in range(5):
        EV.contact_counts(xyz, r, 2.0, ctx=c)
        ms.append(c.kernel_ms('contact_map'))
    t = float(np.median(ms))
    nt = -(-nbead // 64)
    checks = nt * (nt + 1) // 2 * 4096 * S
    res.append({'nbead': nbead, 'nstruct': S, 'kernel_ms': t, 'checks_per_s': checks / t * 1e3,
                'valu_tops': checks * 10 / t / 1e9})
    print(json.dumps(res[-1]), flush=True)
json.dump(res, open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/contact.json', 'w'))
