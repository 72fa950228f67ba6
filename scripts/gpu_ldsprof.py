"""Cycle profile of the LDS anneal kernel (IGM_PROF) on demo-size structures: shader
cycles per MD step for the list builds, the force phase and the rest (calibration for
the domain-decomposed engine) -- tuning only."""
import os
import sys

import numpy as np

os.environ['IGM_PROF'] = '1'
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import mstep_fixtures as F  # noqa: E402
import mstep_stats as MS  # noqa: E402
from igm_amd import _lib, mstep  # noqa: E402
from igm_amd import model as M  # noqa: E402
from igm_amd import synthetic as syn  # noqa: E402

pop, g3 = F.load()
atoms, poly, prm0, chrom = F.demo_model(pop)
n = int(os.environ.get('NS', '256'))
sids = [s % 10 for s in range(n)]
per = [F.hic_bonds_from_golden(g3, atoms.radii, s)[0] for s in sids]
ptr, sb = M.concat_bonds(per)
x = F.struct_major(pop, sids, atoms.n)
proto = MS.scaled_protocol(syn.DEMO_PROTOCOL, float(os.environ.get('SCALE', '0.05')))
prm = M.params_from_cfg({'optimization': {'optimizer_options': proto}}, [((5500.0,) * 3, 1.0)])
seeds = M.lammps_seeds(6535, np.arange(n), 3)
ctx = _lib.context(0)
for rep in range(2):
    xg, ig = mstep.run(prm, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
    p = ctx.mstep_profile()
    ev = max(p['evaluations'], 1)
    print('rep %d anneal %.1f ms; per evaluation (cycles): build %.0f force %.0f rest %.0f; builds/eval %.3f' % (
        rep, ctx.kernel_ms('anneal'), p['build_cycles'] / ev, p['force_cycles'] / ev, p['rest_cycles'] / ev,
        p['builds'] / ev), flush=True)
