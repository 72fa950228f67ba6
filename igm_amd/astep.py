"""A-step (activation-distance assignment) on the MI355X.

Mirrors the reference's A-step call sites:
  * select_pairs       -- ActivationDistanceStep.setup (igm/steps/ActivationDistanceStep.py:111-194):
                          enumerate the .hcs upper triangle in CSR (coo_generator) order, keep
                          intra pairs with p >= intra_sigma and inter pairs with p >= inter_sigma,
                          attach plast from the previous actdist rows.
  * compute_actdist    -- ActivationDistanceStep.task over ALL batches at once
                          (py:196-230) followed by the text round trip of reduce() (py:249):
                          one libigmhip call, rows in CSR pair order.
  * get_actdist        -- the per-pair function signature of the reference (py:336), for
                          callers that use it directly.
No CPU fallback: every result comes from libigmhip.so.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import pair_dtype, row_dtype, result_dtype

actdist_shape = [('row', 'int32'), ('col', 'int32'), ('dist', 'float32'), ('prob', 'float32')]


def copy_index_csr(copy_index, nhap=None):
    """dict {haploid locus: [diploid beads]} (alabtools Index.copy_index) -> CSR arrays."""
    if nhap is None:
        nhap = max(int(k) for k in copy_index) + 1
    ptr = np.zeros(nhap + 1, np.int32)
    idx = []
    for h in range(nhap):
        beads = copy_index.get(h, copy_index.get(str(h), []))
        idx.extend(int(b) for b in beads)
        ptr[h + 1] = len(idx)
    return ptr, np.asarray(idx, np.int32)


def plast_from_rows(rows, n, pi, pj):
    """plast[i, j] of ActivationDistanceStep.setup:144-160: previous actdist rows with
    row < n and col < n, duplicates summed (scipy coo -> lil, in float32)."""
    pl = np.zeros(len(pi), np.float64)
    if rows is None or len(rows) == 0 or len(pi) == 0:
        return pl
    r = np.asarray(rows['row'], np.int64)
    c = np.asarray(rows['col'], np.int64)
    pr = np.asarray(rows['prob'], np.float32)
    ok = (r < n) & (c < n)
    key = r[ok] * n + c[ok]
    val = pr[ok]
    order = np.argsort(key, kind='stable')
    key = key[order]
    val = val[order]
    ukey, start = np.unique(key, return_index=True)
    sums = np.add.reduceat(val, start).astype(np.float32) if len(val) else val
    q = np.asarray(pi, np.int64) * n + np.asarray(pj, np.int64)
    pos = np.searchsorted(ukey, q)
    pos = np.minimum(pos, max(len(ukey) - 1, 0))
    hit = (len(ukey) > 0) & (ukey[pos] == q) if len(ukey) else np.zeros(len(q), bool)
    pl[hit] = sums[pos[hit]].astype(np.float64)
    return pl


def select_pairs(indptr, indices, data, chrom, intra_sigma, inter_sigma, last_rows=None):
    """ActivationDistanceStep.setup:166-177 vectorised.  `indptr/indices/data` are the
    .hcs 'matrix' group (upper triangle, CSR), `chrom` the haploid index chrom.
    A sigma of False/None disables that class, like the reference."""
    indptr = np.asarray(indptr, np.int64)
    n = len(indptr) - 1
    i = np.repeat(np.arange(n, dtype=np.int32), np.diff(indptr))
    j = np.asarray(indices, np.int32)
    p = np.asarray(data, np.float32)
    chrom = np.asarray(chrom)
    same = chrom[i] == chrom[j]
    keep = np.zeros(len(i), bool)
    if intra_sigma is not None and intra_sigma is not False:
        keep |= same & (p.astype(np.float64) >= float(intra_sigma))
    if inter_sigma is not None and inter_sigma is not False:
        keep |= (~same) & (p.astype(np.float64) >= float(inter_sigma))
    pairs = np.zeros(int(keep.sum()), pair_dtype)
    pairs['i'] = i[keep]
    pairs['j'] = j[keep]
    pairs['pwish'] = p[keep].astype(np.float64)
    pairs['plast'] = plast_from_rows(last_rows, n, pairs['i'], pairs['j'])
    return pairs


def _is_device(a):
    return hasattr(a, 'is_cuda') and a.is_cuda


def compute_actdist(xyz, radii, copy_ptr, copy_idx, chrom, pairs, contact_range=2.0, it_corr=1,
                    device=0, return_per_pair=False, ctx=None):
    """Activation distances for every pair (one GPU call).

    xyz: (nbead, nstruct, 3) float32, bead-major (the .hss layout) -- numpy (host)
         or a torch tensor already on the GPU (then every array must be a device tensor
         and the rows come back as a device buffer described by (rows_tensor, n)).
    Returns a structured array with the actdist.hdf5 fields (row, col, dist, prob),
    and the per-pair results when return_per_pair.
    """
    c = ctx or _lib.context(device)
    if _is_device(xyz):
        return _compute_actdist_device(c, xyz, radii, copy_ptr, copy_idx, chrom, pairs, contact_range,
                                       it_corr, return_per_pair)
    xyz = np.ascontiguousarray(xyz, np.float32)
    assert xyz.ndim == 3 and xyz.shape[2] == 3, 'xyz must be (nbead, nstruct, 3)'
    radii = np.ascontiguousarray(radii, np.float32)
    copy_ptr = np.ascontiguousarray(copy_ptr, np.int32)
    copy_idx = np.ascontiguousarray(copy_idx, np.int32)
    chrom = np.ascontiguousarray(chrom, np.int32)
    pairs = np.ascontiguousarray(pairs, pair_dtype)
    nbead, S = xyz.shape[0], xyz.shape[1]
    nhap = len(copy_ptr) - 1
    assert radii.shape[0] == nbead and chrom.shape[0] >= nhap and copy_idx.shape[0] >= copy_ptr[-1]
    assert copy_idx.size == 0 or (copy_idx.min() >= 0 and copy_idx.max() < nbead)
    res = np.zeros(len(pairs), result_dtype)
    # capacity: every pair's maximum row count
    na = np.diff(copy_ptr)
    if len(pairs):
        ni = na[pairs['i']]
        nj = na[pairs['j']]
        same = chrom[pairs['i']] == chrom[pairs['j']]
        cap = int(np.where(same, np.minimum(ni, nj), ni * nj).sum())
    else:
        cap = 0
    rows = np.zeros(max(cap, 1), row_dtype)
    nout = ctypes.c_int64(0)
    rc = c.lib.igm_astep_actdist(c.h, 0, xyz.ctypes.data, nbead, S, radii.ctypes.data, copy_ptr.ctypes.data,
                                 copy_idx.ctypes.data, nhap, chrom.ctypes.data, pairs.ctypes.data, len(pairs),
                                 float(contact_range), int(it_corr), res.ctypes.data, rows.ctypes.data, cap,
                                 ctypes.byref(nout))
    c.check(rc, 'igm_astep_actdist')
    rows = rows[:nout.value]
    if return_per_pair:
        return rows, res
    return rows


def _compute_actdist_device(c, xyz, radii, copy_ptr, copy_idx, chrom, pairs, contact_range, it_corr,
                            return_per_pair):
    import torch
    dev = xyz.device
    nbead, S = int(xyz.shape[0]), int(xyz.shape[1])
    nhap = int(copy_ptr.shape[0]) - 1
    npairs = int(pairs.shape[0]) // pair_dtype.itemsize if pairs.dtype == torch.uint8 else int(pairs.shape[0])
    res = torch.empty(npairs * result_dtype.itemsize, dtype=torch.uint8, device=dev)
    cap = int(npairs) * 4 if npairs else 1
    rows = torch.empty(cap * row_dtype.itemsize, dtype=torch.uint8, device=dev)
    nout = ctypes.c_int64(0)
    c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    try:
        rc = c.lib.igm_astep_actdist(c.h, _lib.IGM_DEVICE_PTRS, _lib.ptr(xyz), nbead, S, _lib.ptr(radii),
                                     _lib.ptr(copy_ptr), _lib.ptr(copy_idx), nhap, _lib.ptr(chrom),
                                     _lib.ptr(pairs), npairs, float(contact_range), int(it_corr),
                                     _lib.ptr(res), _lib.ptr(rows), cap, ctypes.byref(nout))
        c.check(rc, 'igm_astep_actdist')
    finally:
        c.set_stream(None)
    if return_per_pair:
        return rows, nout.value, res
    return rows, nout.value


def get_actdist(i, j, pwish, plast, hss, it_corr, contactRange=2, option=0):
    """Per-pair signature of the reference (ActivationDistanceStep.py:336).  `hss` needs
    get_nstruct(), get_index().copy_index/.chrom, get_radii(), get_bead_crd(k) --
    the same duck type the reference uses.  Returns [(i0, i1, ad, p), ...] with the
    f64 ad/p of the reference (before the task() text formatting)."""
    if option != 0:
        raise NotImplementedError('option=1 is not coded in the reference either (py:357-359)')
    if i == j:
        return []
    idx = hss.get_index()
    copy_index = idx.copy_index
    beads = sorted(set(int(b) for b in list(copy_index[i]) + list(copy_index[j])))
    remap = {b: k for k, b in enumerate(beads)}
    xyz = np.stack([np.asarray(hss.get_bead_crd(b), np.float32) for b in beads])
    radii = np.asarray(hss.get_radii(), np.float32)[beads]
    ptr = np.array([0, len(copy_index[i]), len(copy_index[i]) + len(copy_index[j])], np.int32)
    cidx = np.array([remap[int(b)] for b in copy_index[i]] + [remap[int(b)] for b in copy_index[j]], np.int32)
    ch = np.array([idx.chrom[i], idx.chrom[j]], np.int32)
    pr = np.zeros(1, pair_dtype)
    pr['i'], pr['j'], pr['pwish'], pr['plast'] = 0, 1, pwish, plast
    rows, res = compute_actdist(xyz, radii, ptr, cidx, ch, pr, contactRange, it_corr, return_per_pair=True)
    if res['nrows'][0] == 0:
        return []
    ad, p = float(res['ad'][0]), float(res['p'][0])
    ii, jj = list(copy_index[i]), list(copy_index[j])
    if idx.chrom[i] == idx.chrom[j]:
        return [(i0, i1, ad, p) for i0, i1 in zip(ii, jj)]
    return [(i0, i1, ad, p) for i0 in ii for i1 in jj]
