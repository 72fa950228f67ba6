"""Domain-decomposed engine vs the population engine vs the fp64 oracle on the 200 kb
model (tuning / bring-up; the parity proper is in tests/).  Prints one line per check."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import oracle  # noqa: E402
import mstep_fixtures as F  # noqa: E402
import mstep_stats as MS  # noqa: E402
from igm_amd import _lib, mstep  # noqa: E402
from igm_amd import model as M  # noqa: E402
from igm_amd import synthetic as syn  # noqa: E402


def model200(n, nlocal=15000, nlong=1500, seed=31):
    pop = syn.population_200kb(n, first_sid=500)
    atoms = M.Atoms(pop['radii'])
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    x = np.zeros((n, atoms.n, 3), np.float32)
    x[:, :atoms.nbead] = pop['xyz']
    per = [MS.random_contacts(atoms.radii, atoms.nbead, nlocal, nlong, seed + s) for s in range(n)]
    ptr, sb = M.concat_bonds(per)
    return atoms, poly, ptr, sb, x


def dd(prm):
    p = _lib.MStepParams.from_buffer_copy(prm)
    p.flags |= _lib.IGM_MSTEP_ENGINE_DD
    return p


def main():
    ctx = _lib.context(0)
    n = int(os.environ.get('NS', '2'))
    atoms, poly, ptr, sb, x = model200(n)
    prm = M.params_from_cfg({'optimization': {'optimizer_options': F.DEMO_PROTOCOL}}, [((5500.0,) * 3, 1.0)])
    rng = np.random.default_rng(3)
    xr = x.copy()
    xr[:, :atoms.nbead] += rng.normal(0, 30.0, (n, atoms.nbead, 3)).astype(np.float32)
    fo, _ = oracle.mstep_forces(prm, xr, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2)
    fd, _ = mstep.forces(dd(prm), xr, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, f32=True)
    print('forces dd stats', ctx.engine_stats(), flush=True)
    fp, _ = mstep.forces(prm, xr, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, f32=True)
    print('forces pop stats', ctx.engine_stats(), flush=True)
    nrm = np.linalg.norm(np.linalg.norm(fo, axis=2))
    for nm, fg in (('dd', fd), ('pop', fp)):
        err = np.linalg.norm(np.linalg.norm(fg - fo, axis=2)) / nrm
        print('forces %-4s rel-err vs oracle %.3e  max|dF| %.3e' % (nm, err, np.abs(fg - fo).max()), flush=True)
    v = np.stack([oracle.velocity_create(atoms.flags, 50.0, 21 + s) for s in range(n)]).astype(np.float32)
    xo, _ = oracle.mstep_md(prm, xr.astype(np.float64), v.astype(np.float64), atoms.radii, atoms.flags, poly, ptr,
                            sb, 0.5, 1.2, 50.0, 40.0, 1000.0, 10)
    moved = np.abs(xo - xr).max()
    for nm, pp in (('dd', dd(prm)), ('pop', prm)):
        xg, _ = mstep.md(pp, xr, v, atoms.radii, atoms.flags, poly, ptr, sb, 0.5, 1.2, 50.0, 40.0, 1000.0, 10)
        print('md10 %-4s max|dx| vs oracle %.3e (moved %.1f) stats %s' % (nm, np.abs(xg - xo).max(), moved,
                                                                         ctx.engine_stats()), flush=True)
    scale = float(os.environ.get('SCALE', '0.02'))
    proto = MS.scaled_protocol(syn.DEMO_PROTOCOL, scale)
    prm2 = M.params_from_cfg({'optimization': {'optimizer_options': proto}}, [((5500.0,) * 3, 1.0)])
    seeds = M.lammps_seeds(6535, np.arange(500, 500 + n), 3)
    res = {}
    for nm, pp in (('dd', dd(prm2)), ('dd2', dd(prm2)), ('pop', prm2)):
        t0 = time.time()
        xg, ig = mstep.run(pp, x, atoms.radii, atoms.flags, poly, ptr, sb, seeds)
        dt = time.time() - t0
        res[nm] = (xg, ig)
        print('run x%.2f %-4s %.2f s anneal %.1f ms  E/bead med %.4g  rebuilds %s  stats %s' % (
            scale, nm, dt, ctx.kernel_ms('anneal'), np.median(ig['final_energy']) / atoms.nbead,
            ig['nrebuild'][:4], ctx.engine_stats()), flush=True)
    print('dd rerun bitwise:', np.array_equal(res['dd'][0], res['dd2'][0]), flush=True)


if __name__ == '__main__':
    main()
