"""ORACLE -- test infrastructure only.

CPU restatements of the reference's hot path (see the headers of
actdist_ref.c / mstep_ref.c for the reference file:line each follows).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package; the product (igm_amd) never does.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, 'liboracle.so')

pair_dtype = np.dtype([('i', '<i4'), ('j', '<i4'), ('pwish', '<f8'), ('plast', '<f8')])
row_dtype = np.dtype([('row', '<i4'), ('col', '<i4'), ('dist', '<f4'), ('prob', '<f4')])
result_dtype = np.dtype([('ad', '<f8'), ('p', '<f8'), ('pnow', '<f8'), ('o', '<i4'), ('nrows', '<i4')])

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.check_call(['make', '-C', HERE, '-s'])
        _lib = ctypes.CDLL(LIB)
        _lib.oracle_actdist.restype = ctypes.c_int64
        _lib.oracle_actdist.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]
    return _lib


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def actdist(xyz, radii, copy_ptr, copy_idx, chrom, pairs, contact_range=2.0, it_corr=1, nthreads=1):
    """Reference-semantics A-step on the CPU.  Returns (rows, per_pair)."""
    xyz = _c(xyz, np.float32)
    radii = _c(radii, np.float32)
    copy_ptr = _c(copy_ptr, np.int32)
    copy_idx = _c(copy_idx, np.int32)
    chrom = _c(chrom, np.int32)
    pairs = np.ascontiguousarray(pairs, dtype=pair_dtype)
    nbead, S = xyz.shape[0], xyz.shape[1]
    res = np.zeros(len(pairs), result_dtype)
    L = lib()
    args = [xyz.ctypes.data, nbead, S, radii.ctypes.data, copy_ptr.ctypes.data, copy_idx.ctypes.data,
            len(copy_ptr) - 1, chrom.ctypes.data, pairs.ctypes.data, len(pairs), float(contact_range),
            int(it_corr), res.ctypes.data]
    total = L.oracle_actdist(*(args + [None, 0, int(nthreads)]))
    rows = np.zeros(total, row_dtype)
    L.oracle_actdist(*(args + [rows.ctypes.data, total, int(nthreads)]))
    return rows, res


# ---------------------------------------------------------------- M-step
def _mlib():
    L = lib()
    if not hasattr(L, '_mstep_bound'):
        vp, i32, i64, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
        L.oracle_mstep_run.restype = ctypes.c_int
        L.oracle_mstep_run.argtypes = [vp, i32, i32, vp, vp, vp, vp, i64, vp, vp, vp, vp, vp, i32]
        L.oracle_mstep_run_sf.restype = ctypes.c_int
        L.oracle_mstep_run_sf.argtypes = [vp, i32, i32, vp, vp, vp, i64, vp, i64, vp, vp, vp, vp, vp, i32]
        L.oracle_mstep_forces.restype = ctypes.c_int
        L.oracle_mstep_forces.argtypes = [vp, i32, i32, vp, vp, vp, vp, i64, vp, vp, f64, f64, vp, vp]
        L.oracle_mstep_md.restype = ctypes.c_int
        L.oracle_mstep_md.argtypes = [vp, i32, i32, vp, vp, vp, vp, vp, i64, vp, vp, f64, f64, f64, f64, f64, i32, i32]
        L.oracle_velocity_create.restype = ctypes.c_int
        L.oracle_velocity_create.argtypes = [i32, vp, f64, i32, vp]
        L.oracle_hic_select.restype = ctypes.c_int
        L.oracle_hic_select.argtypes = [i32, i32, vp, vp, vp, vp, vp, i64, vp]
        L._mstep_bound = True
    return L


def _bonds(shared, sptr, sbonds, nstruct):
    from igm_amd._lib import bond_dtype
    shared = np.ascontiguousarray(shared if shared is not None else np.zeros(0, bond_dtype), bond_dtype)
    if sbonds is None:
        sptr = np.zeros(nstruct + 1, np.int64)
        sbonds = np.zeros(1, bond_dtype)
    return shared, np.ascontiguousarray(sptr, np.int64), np.ascontiguousarray(sbonds, bond_dtype)


def mstep_run(params, xyz, radii, flags, shared, sptr, sbonds, seeds, nthreads=1):
    """Full protocol (anneal + CG) per structure in fp64.  xyz (S, N, 3) f32 is
    updated in place (rounded to f32); returns (info, x64).  flags (N,) shared or
    (S, N) one row per structure."""
    import ctypes as C
    from igm_amd._lib import optinfo_dtype
    xyz = np.ascontiguousarray(xyz, np.float32)
    S, N = xyz.shape[0], xyz.shape[1]
    shared, sptr, sbonds = _bonds(shared, sptr, sbonds, S)
    info = np.zeros(S, optinfo_dtype)
    x64 = np.zeros((S, N, 3), np.float64)
    radii = _c(radii, np.float32)
    flags = _c(flags, np.uint32)
    seeds = _c(seeds, np.int32)
    assert flags.shape[-1] == N and (flags.ndim == 1 or flags.shape[0] == S)
    _mlib().oracle_mstep_run_sf(C.byref(params), S, N, xyz.ctypes.data, radii.ctypes.data, flags.ctypes.data,
                                N if flags.ndim == 2 else 0, shared.ctypes.data, len(shared), sptr.ctypes.data,
                                sbonds.ctypes.data, seeds.ctypes.data, info.ctypes.data, x64.ctypes.data,
                                int(nthreads))
    return xyz, info, x64


_vol_keep = []


def set_volume(vol):
    """The map used by IGM_ENV_VOLUME envelopes in later oracle calls (None clears).
    vol: dict(body_idx, nvoxel, origin, grid, matrice (nx, ny, nz, 4) int32)."""
    import ctypes as C
    L = lib()
    L.oracle_set_volume.restype = C.c_int
    L.oracle_set_volume.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    del _vol_keep[:]
    if vol is None:
        L.oracle_set_volume(0, None, None, None, None)
        return
    n = np.ascontiguousarray(vol['nvoxel'], np.int32)
    o = np.ascontiguousarray(vol['origin'], np.float32)
    g = np.ascontiguousarray(vol['grid'], np.float32)
    m = np.ascontiguousarray(vol['matrice'], np.int32)
    _vol_keep.extend([n, o, g, m])
    L.oracle_set_volume(int(vol['body_idx']), n.ctypes.data, o.ctypes.data, g.ctypes.data, m.ctypes.data)


def mstep_forces(params, xyz, radii, flags, shared, sptr, sbonds, evf, envf):
    import ctypes as C
    xyz = np.ascontiguousarray(xyz, np.float32)
    S, N = xyz.shape[0], xyz.shape[1]
    shared, sptr, sbonds = _bonds(shared, sptr, sbonds, S)
    f = np.zeros((S, N, 3), np.float64)
    e = np.zeros((S, 7), np.float64)
    radii = _c(radii, np.float32)
    flags = _c(flags, np.uint32)
    _mlib().oracle_mstep_forces(C.byref(params), S, N, xyz.ctypes.data, radii.ctypes.data, flags.ctypes.data,
                                shared.ctypes.data, len(shared), sptr.ctypes.data, sbonds.ctypes.data,
                                float(evf), float(envf), f.ctypes.data, e.ctypes.data)
    return f, e


def mstep_md(params, x, v, radii, flags, shared, sptr, sbonds, evf, envf, t0, t1, xmax, nsteps, nthreads=1):
    import ctypes as C
    x = np.array(x, np.float64, order='C')
    v = np.array(v, np.float64, order='C')
    S, N = x.shape[0], x.shape[1]
    shared, sptr, sbonds = _bonds(shared, sptr, sbonds, S)
    radii = _c(radii, np.float32)
    flags = _c(flags, np.uint32)
    _mlib().oracle_mstep_md(C.byref(params), S, N, x.ctypes.data, v.ctypes.data, radii.ctypes.data,
                            flags.ctypes.data, shared.ctypes.data, len(shared), sptr.ctypes.data,
                            sbonds.ctypes.data, float(evf), float(envf), float(t0), float(t1), float(xmax),
                            int(nsteps), int(nthreads))
    return x, v


def velocity_create(flags, t, seed):
    flags = _c(flags, np.uint32)
    v = np.zeros((len(flags), 3), np.float64)
    _mlib().oracle_velocity_create(len(flags), flags.ctypes.data, float(t), int(seed), v.ctypes.data)
    return v


def hic_select(xyz, chrom, row, col, dist):
    """(S, n_act) uint8 selection: 1 inter bond, 2 intra bond."""
    xyz = np.ascontiguousarray(xyz, np.float32)
    S, N = xyz.shape[0], xyz.shape[1]
    chrom = _c(chrom, np.int32)
    row = _c(row, np.int32)
    col = _c(col, np.int32)
    dist = _c(dist, np.float32)
    out = np.zeros((S, len(row)), np.uint8)
    _mlib().oracle_hic_select(S, N, xyz.ctypes.data, chrom.ctypes.data, row.ctypes.data, col.ctypes.data,
                              dist.ctypes.data, len(row), out.ctypes.data)
    return out


def violations(vs, tol):
    """ModelingStep.task violation record (py:542-554): histogram of 100 bins on
    [0, 1] + overflow (get_violation_histogram, py:859-869)."""
    vs = np.asarray(vs, np.float64)
    over = np.count_nonzero(vs > 1)
    inner = vs[vs <= 1]
    H, _ = np.histogram(inner, bins=100, range=(0, 1))
    return {'counts': np.concatenate([H, [over]]).tolist(), 'violated_restr': int(np.count_nonzero(vs)),
            'n_violations': int(np.count_nonzero(vs > tol))}


def ranpark_state(seed, n):
    L = _mlib()
    L.oracle_ranpark_state.restype = ctypes.c_int32
    L.oracle_ranpark_state.argtypes = [ctypes.c_int32, ctypes.c_int64]
    return L.oracle_ranpark_state(int(seed), int(n))
