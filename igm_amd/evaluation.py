"""Hi-C evaluation of a population (the GPU contact map of
HicEvaluationStep).

  contact_counts   -- the population contact counts behind HssFile.buildContactMap
                      (igm/steps/HicEvaluationStep.py:109) in one launch
                      (igm_contact_map): counts[i, j] = #structures with
                      |x_i - x_j| <= fl32(contact_range * fl32(r_i + r_j)).
  contact_map      -- reduce()'s output matrix (:108-113): counts / nstruct at
                      contactRange = contact_range * (1 + EPS), copies summed
                      (sumCopies) on the device (igm_contact_map_haploid: no
                      (nbead, nbead) matrix on the host) and clipped to [0, 1].
  hic_evaluation   -- reduce()'s score (:145-179): over the input pairs i != j with
                      p >= sigma that the output matrix stores (non-zero), the mean
                      absolute relative difference, plus the averages stats.txt holds.

buildContactMap and sumCopies live in alabtools, which is not in the reference tree
nor importable here: the contact test restated is IGM's own Hi-C contact (float32 norm
of inter_hic.py:47 against the HarmonicUpperBound r0 of restraints/hic.py), and the copy
sum is the plain sum over copy pairs.  Parity of those two is unpinned; the score
arithmetic follows HicEvaluationStep.reduce line by line.  The comparison is '<=' (a
contact is a satisfied HarmonicUpperBound, inter_hic.py); the commented-out task of
HicEvaluationStep.py:89-91 writes a strict '<'.  The two differ only for a distance
exactly equal to the bound (test_evaluation.py's near-tie case pins which side each
split decision falls on).
"""
import numpy as np

from . import _lib

EPS = 0.05  # HicEvaluationStep.py:22


def contact_counts(xyz, radii, contact_range, ctx=None, device=0):
    """xyz (nbead, S, 3) float32 bead-major (.hss 'coordinates'), radii (nbead,).
    Returns (nbead, nbead) int32, symmetric, diagonal included."""
    c = ctx or _lib.context(device)
    xyz = np.ascontiguousarray(xyz, np.float32)
    radii = np.ascontiguousarray(radii, np.float32)
    if xyz.ndim != 3 or xyz.shape[2] != 3 or radii.shape != (xyz.shape[0],):
        raise ValueError('xyz must be (nbead, nstruct, 3) and radii (nbead,)')
    nbead, S = xyz.shape[0], xyz.shape[1]
    out = np.empty((nbead, nbead), np.int32)
    rc = c.lib.igm_contact_map(c.h, 0, xyz.ctypes.data, nbead, S, radii.ctypes.data, float(contact_range),
                               out.ctypes.data)
    c.check(rc, 'igm_contact_map')
    return out


def haploid_counts(xyz, radii, contact_range, copy_ptr, copy_idx, ctx=None, device=0):
    """The contact counts with the copies summed on the device (igm_contact_map_haploid):
    (nhap, nhap) int32, entry (a, b) = sum of counts[a_k, b_l] over the copies -- no
    (nbead, nbead) intermediate on the host."""
    xyz = np.ascontiguousarray(xyz, np.float32)
    radii = np.ascontiguousarray(radii, np.float32)
    copy_ptr = np.ascontiguousarray(copy_ptr, np.int32)
    copy_idx = np.ascontiguousarray(copy_idx, np.int32)
    if xyz.ndim != 3 or xyz.shape[2] != 3 or radii.shape != (xyz.shape[0],):
        raise ValueError('xyz must be (nbead, nstruct, 3) and radii (nbead,)')
    nbead, S = xyz.shape[0], xyz.shape[1]
    nhap = len(copy_ptr) - 1
    if nhap < 1 or copy_ptr[0] != 0 or np.any(np.diff(copy_ptr) < 0) or copy_ptr[-1] != len(copy_idx) or \
            len(copy_idx) != nbead:
        raise ValueError('copy_ptr must be non-decreasing from 0 to len(copy_idx) == nbead')
    c = ctx or _lib.context(device)
    out = np.empty((nhap, nhap), np.int32)
    rc = c.lib.igm_contact_map_haploid(c.h, 0, xyz.ctypes.data, nbead, S, radii.ctypes.data, float(contact_range),
                                       copy_ptr.ctypes.data, copy_idx.ctypes.data, nhap, out.ctypes.data)
    c.check(rc, 'igm_contact_map_haploid')
    return out


def sum_copies(full, copy_ptr, copy_idx):
    """(nbead, nbead) -> (nhap, nhap): entry (a, b) sums full over the copies of a and b
    (host restatement of sumCopies; small inputs and tests only)."""
    nhap = len(copy_ptr) - 1
    hap_of = np.empty(len(copy_idx), np.int64)
    for a in range(nhap):
        hap_of[copy_idx[copy_ptr[a]:copy_ptr[a + 1]]] = a
    out = np.zeros((nhap, nhap), np.float64)
    np.add.at(out, (hap_of[:, None], hap_of[None, :]), full)
    return out


def contact_map(xyz, radii, contact_range, copy_ptr, copy_idx, ctx=None, device=0):
    """reduce()'s out_matrix: haploid contact frequencies clipped to [0, 1].  The copies
    are summed as integers on the device and divided by nstruct once (the reference
    divides first, then sums float64 copies: equal up to the last bit of the sum)."""
    counts = haploid_counts(xyz, radii, contact_range * (1 + EPS), copy_ptr, copy_idx, ctx=ctx, device=device)
    return np.clip(counts / np.float64(np.asarray(xyz).shape[1]), 0, 1)


def hic_evaluation(input_matrix, output_matrix, sigma):
    """(score, average diff, average relative diff, n pairs) of HicEvaluationStep.reduce
    (:145-179) on dense (nhap, nhap) matrices; the upper triangle is the stored one."""
    inp = np.triu(np.asarray(input_matrix, np.float64), 1)
    out = np.triu(np.asarray(output_matrix, np.float64), 1)
    sel = (inp >= sigma) & (out != 0)
    p, pout = inp[sel], out[sel]
    diffs = pout - p
    reldiffs = diffs / p
    score = float(np.abs(reldiffs).mean()) if len(p) else float('nan')
    return score, float(np.average(diffs)) if len(p) else float('nan'), \
        float(np.average(reldiffs)) if len(p) else float('nan'), int(len(p))
