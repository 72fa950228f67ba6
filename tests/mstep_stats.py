"""Population-level comparison of M-step runs (test helper).

Annealing trajectories are chaotic and RNG-driven: a GPU run (f32 MD) and the fp64
oracle started from identical inputs end in different local minima, so the M-step is
compared the way SURVEY 7 hard part 1(iii) prescribes -- as populations.  A run is
summarised per structure (energies per bead, violation fraction of its restraints,
final Temp, Verlet rebuilds) and two runs are `same_population` when a two-sample
Kolmogorov-Smirnov test does not separate them.  tests/test_mstep_stats.py shows on
the oracle alone that this statistic accepts a reseeded rerun and rejects a 2x bond K
or a 2x soft-pair evfactor, so a convention or precision error of that size in the
GPU path cannot pass it.

Frustration matters: the demo restraint set anneals to E ~ 0 (every restraint
satisfied), where the final state does not depend on K at all.  `random_contacts`
adds Hi-C-like restraints that cannot all be met, so the final energies balance the
bond, soft-pair and envelope terms and respond to each of them.
"""
import json

import numpy as np


def scaled_protocol(protocol, scale):
    """The protocol with every MD step count scaled (all stages, relax and CG kept)."""
    p = json.loads(json.dumps(protocol))
    cap = p['custom_annealing_protocol']
    cap['mdsteps'] = [max(1, int(round(n * scale))) for n in cap['mdsteps']]
    cap['relax']['mdsteps'] = max(1, int(round(cap['relax']['mdsteps'] * scale)))
    return p


def random_contacts(radii, nbead, nlocal, nlong, seed, cr=2.0, k=1.0):
    """Hi-C-like bonds (harmonic upper bound, r0 = cr (r_i + r_j)): nlocal pairs at
    genomic separations 2..60 beads, nlong between random beads."""
    from igm_amd import model as M
    from igm_amd._lib import bond_dtype
    rng = np.random.default_rng(seed)
    i1 = rng.integers(0, nbead - 61, nlocal)
    j1 = i1 + rng.integers(2, 61, nlocal)
    i2 = rng.integers(0, nbead, nlong)
    j2 = rng.integers(0, nbead, nlong)
    i = np.concatenate([i1, i2])
    j = np.concatenate([j1, j2])
    keep = i != j
    b = np.zeros(int(keep.sum()), bond_dtype)
    b['i'], b['j'] = i[keep], j[keep]
    b['r0'] = M.r0_contact(cr, radii[b['i']], radii[b['j']]).astype(np.float32)
    b['k'] = k
    return b


def violation_fraction(x, bonds, tol=0.05):
    """Fraction of upper-bound bonds stretched past (1 + tol) r0 (ModelingStep's
    n_violations / n_imposed for the bond classes, ratio (r - d) / d > tol)."""
    d = np.linalg.norm(x[bonds['i'].astype(np.int64)].astype(np.float64) -
                       x[(bonds['j'] & 0x7fffffff).astype(np.int64)].astype(np.float64), axis=1)
    r0 = bonds['r0'].astype(np.float64)
    return float(np.count_nonzero((d - r0) / r0 > tol)) / max(len(bonds), 1)


def population_stats(info, xyz, shared, ptr, sbonds, nbead):
    """Per-structure summary of a run: dict of arrays (S,)."""
    S = len(info)
    out = {'pair': info['pair_energy'] / nbead, 'bond': info['bond_energy'] / nbead,
           'total': info['final_energy'] / nbead, 'temp': info['temp'].astype(np.float64),
           'rebuilds': info['nrebuild'].astype(np.float64)}
    vf = np.zeros(S)
    for s in range(S):
        b = np.concatenate([shared, sbonds[ptr[s]:ptr[s + 1]]]) if ptr is not None else shared
        vf[s] = violation_fraction(xyz[s], b)
    out['viol_frac'] = vf
    return out


def same_population(a, b, keys=('pair', 'bond', 'total', 'viol_frac'), alpha=1e-3):
    """(ok, {key: KS p-value}): two runs agree when no key separates them at level alpha."""
    from scipy import stats
    pv = {k: float(stats.ks_2samp(a[k], b[k]).pvalue) for k in keys}
    return all(p > alpha for p in pv.values()), pv
