"""Dev check: one MD step of the population engine with and without block windows (IGM_POP_WIN)
on 2 structures of the 200 kb model; prints the largest coordinate/velocity differences."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from igm_amd import model as M, mstep, synthetic as syn  # noqa: E402

pop = syn.population_200kb(2)
atoms = M.Atoms(pop['radii'])
poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
prm = M.params_from_cfg({'optimization': {'optimizer_options': syn.DEMO_PROTOCOL}}, [((5500.0,) * 3, 1.0)])
x = np.zeros((2, atoms.n, 3), np.float32)
x[:, :atoms.nbead] = pop['xyz']
v = mstep.velocity_create(atoms.flags, [11, 12], 50.0)
out = {}
for w in ('0', '1'):
    os.environ['IGM_POP_WIN'] = w
    for n in (1, 2, 20):
        out[(w, n)] = mstep.md(prm, x, v, atoms.radii, atoms.flags, poly, None, None, 1.0, 1.0, 50.0, 40.0, 1000.0, n)
for n in (1, 2, 20):
    a, b = out[('0', n)], out[('1', n)]
    dx = np.abs(a[0] - b[0]).max()
    dv = np.abs(a[1] - b[1]).max()
    nd = int(np.count_nonzero(a[1] != b[1]))
    print('steps %d: max |dx| %.3g, max |dv| %.3g, velocity components differing %d of %d' % (n, dx, dv, nd, a[1].size))
