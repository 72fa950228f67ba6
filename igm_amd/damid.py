"""DamID A-step (lamina activation distances) on the MI355X.

Mirrors igm/steps/DamidActivationDistanceStep.py:
  * select_loci          -- setup() (py:159-221): loci with profile >= sigma, p_exp,
                            plast from the previous damid_actdist rows ({loc: prob}
                            looked up by the haploid locus id, exactly as py:188-189, 213).
  * compute_damid_actdist -- task() over ALL batches in one libigmhip call, followed by
                            the "%6d %.5f %.5f" text round trip of task()/reduce():
                            bit-exact rows {loc, dist, prob}.
  * get_damid_actdist_I  -- the per-locus function signature (py:376).
Shapes 'sphere' and 'ellipsoid' are supported; 'exp_map' (volumetric maps read from
files) is out of scope.  Unlike the reference's task(), the
ellipsoid really is computed (the reference tests `'shape' == 'ellipsoid'`, a string
literal, so an ellipsoid run emits no rows: defect D3, py:258).
No CPU fallback: every row comes from libigmhip.so.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import damid_row_dtype, result_dtype

damid_actdist_shape = [('loc', 'int32'), ('dist', 'float32'), ('prob', 'float32')]
damid_actdist_fmt_str = "%6d %.5f %.5f"
SHAPES = {'sphere': 0, 'ellipsoid': 1, 'exp_map': 2}


def select_loci(profile, sigma, last_rows=None):
    """setup() (py:182-217): (loci int32, p_exp f32, plast f32)."""
    profile = np.asarray(profile, np.float32)
    mask = profile >= np.float32(sigma)
    ii = np.where(mask)[0].astype(np.int32)
    p_exp = profile[mask]
    plast = np.zeros(len(ii), np.float32)
    if last_rows is not None and len(last_rows):
        last_prob = {int(i): p for i, p in zip(last_rows['loc'], last_rows['prob'])}
        plast = np.array([last_prob.get(int(i), 0.) for i in ii], np.float32)
    return ii, p_exp, plast


def _nucleus_param(shape, nucleus_param):
    if shape not in SHAPES:
        raise NotImplementedError('DamID restraint for shape %s has not been implemented yet.' % shape)
    if shape == 'exp_map':
        return np.zeros(3, np.float64)
    if shape == 'sphere':
        return np.array([float(np.ravel(nucleus_param)[0])] * 3, np.float64)
    a = np.asarray(nucleus_param, np.float64).ravel()
    if a.shape != (3,):
        raise ValueError('ellipsoid needs 3 semiaxes')
    return a


def compute_damid_actdist(xyz, radii, copy_ptr, copy_idx, loci, p_exp, plast, it_corr=1, contact_range=0.05,
                          shape='sphere', nucleus_param=5000.0, device=0, return_per_locus=False, ctx=None,
                          volumes=None, struct_map=None):
    """Rows of every selected locus, in locus order (the concatenation of all task()
    batches).  xyz: (nbead, nstruct, 3) float32 bead-major (the .hss layout).
    shape 'exp_map' (get_damid_actdist_exp, py:475-577): `volumes` are the VolumeFile
    maps (igm_amd.volume.read_volume) and struct_map[s] the map of structure s
    (volumes_idx); they are staged into the context."""
    c = ctx or _lib.context(device)
    if shape == 'exp_map':
        from . import volume as V
        if volumes is None:
            raise ValueError('exp_map needs the volume maps')
        V.stage(c, volumes, struct_map)
    xyz = np.ascontiguousarray(xyz, np.float32)
    assert xyz.ndim == 3 and xyz.shape[2] == 3, 'xyz must be (nbead, nstruct, 3)'
    radii = np.ascontiguousarray(radii, np.float32)
    copy_ptr = np.ascontiguousarray(copy_ptr, np.int32)
    copy_idx = np.ascontiguousarray(copy_idx, np.int32)
    loci = np.ascontiguousarray(loci, np.int32)
    p_exp = np.ascontiguousarray(p_exp, np.float32)
    plast = np.ascontiguousarray(plast, np.float32)
    nbead, S = xyz.shape[0], xyz.shape[1]
    nhap = len(copy_ptr) - 1
    assert radii.shape[0] == nbead and len(p_exp) == len(loci) == len(plast)
    assert copy_idx.size == 0 or (copy_idx.min() >= 0 and copy_idx.max() < nbead)
    par = _nucleus_param(shape, nucleus_param)
    ok = (loci >= 0) & (loci < nhap)  # out-of-range loci are rejected by the library
    cap = int(np.diff(copy_ptr)[loci[ok]].sum()) if len(loci) else 0
    rows = np.zeros(max(cap, 1), damid_row_dtype)
    res = np.zeros(len(loci), result_dtype)
    nout = ctypes.c_int64(0)
    rc = c.lib.igm_damid_actdist(c.h, 0, xyz.ctypes.data, nbead, S, radii.ctypes.data, copy_ptr.ctypes.data,
                                 copy_idx.ctypes.data, nhap, loci.ctypes.data, p_exp.ctypes.data,
                                 plast.ctypes.data, len(loci), int(it_corr), float(contact_range), SHAPES[shape],
                                 par.ctypes.data, res.ctypes.data, rows.ctypes.data, cap, ctypes.byref(nout))
    c.check(rc, 'igm_damid_actdist')
    rows = rows[:nout.value]
    if return_per_locus:
        return rows, res
    return rows


def get_damid_actdist_I(I, p_exp, plast, hss, it_corr, contact_range=0.05, shape="sphere", nucleus_param=5000.0):
    """Per-locus signature of the reference (py:376): [(i, ad, p) for i in copies]
    with the float64 ad/p before the text formatting.  `hss` is the reference's duck
    type (get_nstruct, get_index().copy_index, get_radii, get_bead_crd)."""
    copy_index = hss.get_index().copy_index
    ii = [int(b) for b in copy_index[I]]
    xyz = np.stack([np.asarray(hss.get_bead_crd(b), np.float32) for b in ii])
    radii = np.asarray(hss.get_radii(), np.float32)[ii]
    ptr = np.array([0, len(ii)], np.int32)
    cidx = np.arange(len(ii), dtype=np.int32)
    _, res = compute_damid_actdist(xyz, radii, ptr, cidx, [0], [p_exp], [plast], it_corr, contact_range, shape,
                                   nucleus_param, return_per_locus=True)
    p = float(res['p'][0])
    ad = float(res['ad'][0]) if res['o'][0] >= 0 else 2
    return [(i, ad, p) for i in ii]
