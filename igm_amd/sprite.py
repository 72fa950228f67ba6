"""SPRITE A-step (cluster -> structure assignment) on the MI355X.

Mirrors igm/steps/SpriteAssignmentStep.py:
  * cluster_tables -- the per-cluster bookkeeping of compute_gyration_radius
                      (igm/cython_compiled/sprite.pyx:184-283): sorted cluster,
                      single- vs multi-chromosome, segments grouped by chromosome,
                      one representative per chromosome drawn with np.random.choice in
                      the reference's order (so a seeded run draws the same ones),
                      clusters over max_chrom_in_cluster skipped (py:114-121).
  * task          -- SpriteAssignmentStep.task over ALL clusters in one libigmhip call:
                      Rg^2 of every (cluster, structure), the keep_best structures
                      (argpartition + argsort, py:138-143) and their selected beads.
  * assign        -- reduce() (py:173-260): the sequential Gibbs assignment with the
                      occupancy penalty, host-side (it is a serial chain over clusters).
No CPU fallback for the Rg^2 / selection: it comes from libigmhip.so.
"""
import numpy as np

from . import _lib


def cluster_tables(clusters, chrom, copy_ptr, max_chrom_in_cluster=6, rng=None):
    """CSR description of the clusters for igm_sprite_assign.  Regions are the haploid
    loci (alt_ptr/alt_bead = the copy index).  Returns dict(seg_ptr, seg_region,
    seg_rep, rep_ptr, rep_region, kept (indices of computed clusters), sizes)."""
    rng = np.random if rng is None else rng
    chrom = np.asarray(chrom)
    seg_ptr, seg_region, seg_rep, rep_ptr, rep_region, kept = [0], [], [], [0], [], []
    for q, cl in enumerate(clusters):
        cl = np.asarray(cl)
        if len(np.unique(chrom[cl])) > max_chrom_in_cluster:
            continue
        cl = np.sort(cl)
        cch = chrom[cl]
        uch = np.unique(cch)
        if len(uch) == 1:
            seg_region += cl.tolist()
            seg_rep += [-1] * len(cl)
        else:
            by_chrom = [cl[np.where(cch == c)] for c in uch]
            reps = [int(rng.choice(x)) for x in by_chrom if len(x)]
            for slot, segs in enumerate(by_chrom):
                seg_region += segs.tolist()
                seg_rep += [slot] * len(segs)
            rep_region += reps
        seg_ptr.append(len(seg_region))
        rep_ptr.append(len(rep_region))
        kept.append(q)
    i32 = lambda a: np.ascontiguousarray(a, np.int32)
    return dict(seg_ptr=i32(seg_ptr), seg_region=i32(seg_region), seg_rep=i32(seg_rep), rep_ptr=i32(rep_ptr),
                rep_region=i32(rep_region), kept=np.asarray(kept, np.int64))


def rg2_select(xyz, copy_ptr, copy_idx, tables, keep_best, device=0, ctx=None, return_rg2=False):
    """One igm_sprite_assign call over the computed clusters of `tables`.
    Returns best_idx (n, kb) i32, best_rg2 (n, kb) f32, best_sel (flat, cluster c's
    (kb, nseg_c) block at seg_ptr[c]*kb) and optionally rg2 (n, nstruct)."""
    c = ctx or _lib.context(device)
    xyz = np.ascontiguousarray(xyz, np.float32)
    assert xyz.ndim == 3 and xyz.shape[2] == 3, 'xyz must be (nbead, nstruct, 3)'
    copy_ptr = np.ascontiguousarray(copy_ptr, np.int32)
    copy_idx = np.ascontiguousarray(copy_idx, np.int32)
    nbead, S = xyz.shape[0], xyz.shape[1]
    t = tables
    n = len(t['seg_ptr']) - 1
    kb = int(keep_best)
    bi = np.zeros((n, kb), np.int32)
    bv = np.zeros((n, kb), np.float32)
    bs = np.zeros(max(int(t['seg_ptr'][-1]) * kb, 1), np.int32)
    rg2 = np.zeros((n, S), np.float32) if return_rg2 else None
    p = lambda a: a.ctypes.data if len(a) else None
    rc = c.lib.igm_sprite_assign(c.h, 0, xyz.ctypes.data, nbead, S, n, t['seg_ptr'].ctypes.data, p(t['seg_region']),
                                 p(t['seg_rep']), t['rep_ptr'].ctypes.data, p(t['rep_region']), len(copy_ptr) - 1,
                                 copy_ptr.ctypes.data, copy_idx.ctypes.data, kb, _lib.ptr(rg2), bi.ctypes.data,
                                 bv.ctypes.data, bs.ctypes.data)
    c.check(rc, 'igm_sprite_assign')
    if return_rg2:
        return bi, bv, bs, rg2
    return bi, bv, bs


def task(xyz, clusters, chrom, copy_ptr, copy_idx, keep_best=100, max_chrom_in_cluster=6, device=0, ctx=None,
         rng=None):
    """SpriteAssignmentStep.task for all clusters: (indexes, values, selected_beads)
    lists with the reference's per-cluster shapes ((kb,), (kb,), (kb, len(cluster)));
    -1 entries for clusters over max_chrom_in_cluster (py:114-121)."""
    t = cluster_tables(clusters, chrom, copy_ptr, max_chrom_in_cluster, rng)
    bi, bv, bs = rg2_select(xyz, copy_ptr, copy_idx, t, keep_best, device=device, ctx=ctx)
    kb = int(keep_best)
    indexes, values, selected = [], [], []
    pos = {int(q): k for k, q in enumerate(t['kept'])}
    for q, cl in enumerate(clusters):
        k = pos.get(q)
        if k is None:
            selected.append(np.zeros((kb, len(cl)), np.int32) - 1)
            indexes.append(np.array([-1] * kb))
            values.append(np.array([-1] * kb))
            continue
        g0, g1 = int(t['seg_ptr'][k]), int(t['seg_ptr'][k + 1])
        selected.append(bs[g0 * kb:g1 * kb].reshape(kb, g1 - g0))
        indexes.append(bi[k])
        values.append(bv[k])
    return indexes, values, selected


def assign(values, indexes, selected, n_struct, kT=100.0, order=None, rng=None):
    """reduce() (SpriteAssignmentStep.py:173-260) over clusters in `order` (the
    reference walks batches in a random permutation, clusters in batch order):
    Gibbs selection among the keep_best structures with the occupancy penalty.
    Returns (assignment (ncl,) i32, selected beads per cluster)."""
    rng = np.random if rng is None else rng
    ncl = len(values)
    order = range(ncl) if order is None else order
    occupancy = np.zeros(n_struct, dtype=np.int32)
    assignment = np.zeros(ncl, dtype=np.int32)
    aveN = float(ncl) / n_struct
    stdN = np.sqrt(aveN)
    chosen = [None] * ncl
    for ci in order:
        best_rg2s, curr_idx = values[ci], indexes[ci]
        if best_rg2s[0] < 0:
            pos, si = 0, -1
        else:
            best_rgs = np.sqrt(best_rg2s)
            pen = np.clip(occupancy[curr_idx] - aveN, 0., None) / stdN
            E = (best_rgs - best_rgs[0]) / kT + pen
            P = np.cumsum(np.exp(-(E - E[0])))
            e = rng.rand() * P[-1]
            pos = np.searchsorted(P, e, side='left')
            si = curr_idx[pos]
            occupancy[si] += 1
        assignment[ci] = si
        chosen[ci] = selected[ci][pos]
    return assignment, chosen
