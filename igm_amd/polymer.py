"""Polymer-distance A-step and its M-step restraint.

  batches             -- PolymerAssignmentStep.setup (igm/steps/PolymerAssignmentStep.py:
                         55-79): loci 0 .. nbead-2 in batches of 1000 (as there, an nbead
                         that is a multiple of 1000 puts locus nbead-1 in the last batch;
                         assign rejects it where task() raises IndexError).
  assign              -- PolymerAssignmentStep.task (:84-129) for any set of loci in one
                         launch (igm_polymer_assign): the (i, i+1) distances of every
                         structure are ranked and the rank-th smallest of S draws from
                         the bin distribution is assigned.  The draws come from `rng`
                         (a numpy RandomState; default the global one, as the reference)
                         in the reference's order: per locus, the S uniforms of
                         np.random.choice(edges, S, p=prob).  Seeded identically, the
                         output equals the reference's nn_dist bit for bit.
  polymer_distrib_bonds
                      -- PolymerDistrib._apply (igm/restraints/polymer_bis.py:50-90) for a
                         batch of structures: for each locus with i, i+1 on one chromosome
                         a lower bound max(0, t - tol) then an upper bound t + tol.
"""
import numpy as np

from . import _lib
from ._lib import bond_dtype
from .model import LOWER_BOUND_BIT

BATCH_SIZE = 1000  # PolymerAssignmentStep.setup


def batches(nbead, batch_size=BATCH_SIZE):
    """setup()'s argument_list: [(batch_id, range(i, i + batch_size)), ...] over 0..nbead-2."""
    out = []
    for i in range(0, nbead - 1, batch_size):
        out.append((len(out), range(i, nbead - 1) if i + batch_size > nbead else range(i, i + batch_size)))
    return out


def _check_distribution(edges, prob):
    """The argument checks RandomState.choice applies to (a, p) (same errors)."""
    edges = np.asarray(edges)
    prob = np.asarray(prob, np.float64)
    if edges.ndim != 1 or edges.size == 0:
        raise ValueError('a must be 1-dimensional and non-empty')
    if prob.ndim != 1:
        raise ValueError('p must be 1-dimensional')
    if prob.size != edges.size:
        raise ValueError('a and p must have same size')
    if np.isnan(prob).any():
        raise ValueError('probabilities contain NaN')
    if np.any(prob < 0):
        raise ValueError('probabilities are not non-negative')
    if abs(float(np.sum(prob)) - 1.0) > np.sqrt(np.finfo(np.float64).eps):
        raise ValueError('probabilities do not sum to 1')
    return edges.astype(np.float64), np.ascontiguousarray(prob)


def assign(xyz, edges, prob, rng=None, loci=None, return_dists=False, chunk=BATCH_SIZE, ctx=None, device=0):
    """xyz (nbead, S, 3) float32 bead-major (the .hss 'coordinates').  Returns (loci int32,
    nn_dist (nloci, S) float32[, dists (nloci, S) float32]).  `chunk` loci per launch
    bounds the host memory of the draws (8 B per locus and structure)."""
    c = ctx or _lib.context(device)
    xyz = np.ascontiguousarray(xyz, np.float32)
    nbead, S = xyz.shape[0], xyz.shape[1]
    e, p = _check_distribution(edges, prob)
    loci = np.arange(nbead - 1, dtype=np.int32) if loci is None else np.ascontiguousarray(loci, np.int32)
    rng = np.random.mtrand._rand if rng is None else rng
    out = np.zeros((len(loci), S), np.float32)
    dist = np.zeros((len(loci), S), np.float32) if return_dists else None
    chunk = max(1, int(chunk))
    for q0 in range(0, len(loci), chunk):
        lq = loci[q0:q0 + chunk]
        u = np.ascontiguousarray(rng.random_sample((len(lq), S)))  # one choice() per locus, in order
        o = out[q0:q0 + len(lq)]
        dd = dist[q0:q0 + len(lq)] if return_dists else None
        rc = c.lib.igm_polymer_assign(c.h, 0, xyz.ctypes.data, nbead, S, lq.ctypes.data, len(lq), u.ctypes.data,
                                      len(e), e.ctypes.data, p.ctypes.data, o.ctypes.data,
                                      dd.ctypes.data if dd is not None else None)
        c.check(rc, 'igm_polymer_assign')
    return (loci, out, dist) if return_dists else (loci, out)


def polymer_distrib_bonds(loci, nn_dist, chrom, struct_ids, tolerance=10.0, kspring=2.0):
    """PolymerDistrib._apply for the structures struct_ids: list of igm_bond arrays, in
    the reference's force order (per locus: lower bound, then upper bound)."""
    loci = np.asarray(loci, np.int64)
    chrom = np.asarray(chrom)
    keep = chrom[loci] == chrom[loci + 1]
    li = loci[keep]
    nn = np.asarray(nn_dist, np.float32)[keep]
    tol = float(tolerance)
    out = []
    for sid in struct_ids:
        t = nn[:, int(sid)].astype(np.float64)  # float32 target op Python float: float64 (NumPy 1.x)
        n = len(li)
        b = np.zeros(2 * n, bond_dtype)
        b['i'][0::2] = li
        b['i'][1::2] = li
        b['j'][0::2] = (li + 1).astype(np.uint32) | LOWER_BOUND_BIT
        b['j'][1::2] = li + 1
        b['r0'][0::2] = np.maximum(0.0, t - tol)  # max(0, target_dist - tol)
        b['r0'][1::2] = t + tol
        b['k'] = float(kspring)
        out.append(b)
    return out
