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
import numpy as np

from igm_amd.workloads import random_contacts, scaled_protocol  # noqa: E402,F401  (shared with the bench)


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
