"""A/B bitwise check of two libigmhip builds on the population engine (tuning aid):
python scripts/ab_md_equal.py OUT.npy  -- runs a 200 kb MD segment with list rebuilds
through the library IGM_HIP_LIB names and saves (x, v); compare two outputs with --cmp A B."""
import sys

import numpy as np

sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
if sys.argv[1] == '--cmp':
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    print('bitwise equal' if np.array_equal(a, b) else 'DIFFER max %.3g' % np.abs(a - b).max())
    sys.exit(0 if np.array_equal(a, b) else 1)
import oracle
from igm_amd import model as M, mstep, synthetic as syn

pop = syn.population_200kb(4)
atoms = M.Atoms(pop['radii'])
poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
prm = M.params_from_cfg({'optimization': {'optimizer_options': syn.DEMO_PROTOCOL}}, [((5500.0,) * 3, 1.0)])
x = np.zeros((4, atoms.n, 3), np.float32)
x[:, :atoms.nbead] = pop['xyz']
rng = np.random.default_rng(9)
per = []
for s in range(4):
    i = rng.integers(0, atoms.nbead, 4000)
    j = (i + rng.integers(2, 60, 4000)) % atoms.nbead
    b = np.zeros(4000, poly.dtype)
    b['i'], b['j'] = i, j
    b['r0'] = M.r0_contact(2.0, atoms.radii[i], atoms.radii[j]).astype(np.float32)
    b['k'] = 1.0
    per.append(b)
ptr, sb = M.concat_bonds(per)
v = np.stack([oracle.velocity_create(atoms.flags, 2000.0, 31 + s) for s in range(4)]).astype(np.float32)
xo, vo = mstep.md(prm, x, v, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, 2000.0, 1500.0, 1000.0, 200)
np.save(sys.argv[1], np.stack([xo, vo]))
print('moved %.1f' % np.abs(xo - x).max())
