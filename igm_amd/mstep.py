"""M-step on the MI355X: batched replacement of the serial-LAMMPS kernel.

Reference call chain replaced (one structure per process there, the whole
population per call here):
  ModelingStep.task          igm/steps/ModelingStep.py:164-573
    interHiC/intraHiC._apply restraints/inter_hic.py:294-312   -> hic_select (GPU)
    model.optimize(cfg)      model/model.py:130-137
      lammps.optimize        model/kernel/lammps.py:361-492      -> run (GPU anneal + CG)
    violation statistics     ModelingStep.py:511-557,859-869     -> violations (GPU)

Every function here is a thin wrapper over libigmhip.so (include/igm_hip.h).
Arrays may be numpy (host) or torch tensors resident on the GPU (then all of
them must be; pass device=True semantics by giving tensors).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import IGM_DEVICE_PTRS, IGM_F32_PATH, bond_dtype, optinfo_dtype
from . import model as M

REC = 104  # counts[101], violated_restr, n_violations, n_imposed


def _is_dev(a):
    return hasattr(a, 'is_cuda') and a.is_cuda


def _np(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _prm(params, flags):
    """params with IGM_MSTEP_STRUCT_FLAGS set when flags has one row per structure."""
    nd = flags.dim() if hasattr(flags, 'dim') else np.ndim(flags)
    if nd != 2:
        return params
    p = _lib.MStepParams.from_buffer_copy(params)
    p.flags |= _lib.IGM_MSTEP_STRUCT_FLAGS
    return p


def _bonds_args(shared, sptr, sbonds, nstruct):
    shared = _np(shared if shared is not None else np.zeros(0, bond_dtype), bond_dtype)
    if sbonds is None or sptr is None:
        return shared, None, None
    return shared, _np(sptr, np.int64), _np(sbonds, bond_dtype)


def run(params, xyz, radii, flags, shared_bonds, sbond_ptr, sbonds, seeds, ctx=None, device=0):
    """Anneal + CG for every structure.  xyz (S, N, 3) float32 struct-major.
    Returns (xyz_out, info).  With torch device tensors everything stays on the GPU
    and xyz is updated in place."""
    c = ctx or _lib.context(device)
    if _is_dev(xyz):
        import torch
        S, N = int(xyz.shape[0]), int(xyz.shape[1])
        info = torch.empty(S * optinfo_dtype.itemsize, dtype=torch.uint8, device=xyz.device)
        c.set_stream(torch.cuda.current_stream(xyz.device).cuda_stream)
        prm = _prm(params, flags)
        try:
            rc = c.lib.igm_mstep_run(c.h, IGM_DEVICE_PTRS, ctypes.byref(prm), S, N, _lib.ptr(xyz),
                                     _lib.ptr(radii), _lib.ptr(flags), _lib.ptr(shared_bonds),
                                     int(shared_bonds.shape[0]) // bond_dtype.itemsize
                                     if shared_bonds.dtype == torch.uint8 else int(shared_bonds.shape[0]),
                                     _lib.ptr(sbond_ptr), _lib.ptr(sbonds), _lib.ptr(seeds), _lib.ptr(info))
            c.check(rc, 'igm_mstep_run')
        finally:
            c.set_stream(None)
        return xyz, info
    xyz = np.array(xyz, dtype=np.float32, order='C', copy=True)
    S, N = xyz.shape[0], xyz.shape[1]
    radii = _np(radii, np.float32)
    flags = _np(flags, np.uint32)
    seeds = _np(seeds, np.int32)
    shared, sptr, sb = _bonds_args(shared_bonds, sbond_ptr, sbonds, S)
    assert radii.shape[0] == N and flags.shape[-1] == N and seeds.shape[0] == S
    assert flags.ndim == 1 or flags.shape[0] == S, 'per-structure flags must be (S, N)'
    prm = _prm(params, flags)
    info = np.zeros(S, optinfo_dtype)
    rc = c.lib.igm_mstep_run(c.h, 0, ctypes.byref(prm), S, N, xyz.ctypes.data, radii.ctypes.data,
                             flags.ctypes.data, shared.ctypes.data if len(shared) else None, len(shared),
                             _lib.ptr(sptr), _lib.ptr(sb), seeds.ctypes.data, info.ctypes.data)
    c.check(rc, 'igm_mstep_run')
    return xyz, info


def forces(params, xyz, radii, flags, shared_bonds, sbond_ptr, sbonds, evf, envf, f32=False, ctx=None, device=0):
    """Forces (S, N, 3) and energies (S, 7) = {total, pair, bond, env0..3} (parity harness)."""
    c = ctx or _lib.context(device)
    xyz = _np(xyz, np.float32)
    S, N = xyz.shape[0], xyz.shape[1]
    shared, sptr, sb = _bonds_args(shared_bonds, sbond_ptr, sbonds, S)
    f = np.zeros((S, N, 3), np.float32)
    e = np.zeros((S, 7), np.float64)
    prm = _prm(params, flags)
    rc = c.lib.igm_mstep_forces(c.h, IGM_F32_PATH if f32 else 0, ctypes.byref(prm), S, N, xyz.ctypes.data,
                                _np(radii, np.float32).ctypes.data, _np(flags, np.uint32).ctypes.data,
                                shared.ctypes.data if len(shared) else None, len(shared), _lib.ptr(sptr),
                                _lib.ptr(sb), float(evf), float(envf), f.ctypes.data, e.ctypes.data)
    c.check(rc, 'igm_mstep_forces')
    return f, e


def md(params, xyz, v, radii, flags, shared_bonds, sbond_ptr, sbonds, evf, envf, t0, t1, xmax, nsteps,
       ctx=None, device=0):
    """One 'run nsteps' segment (nve/limit + temp/rescale) from given velocities."""
    c = ctx or _lib.context(device)
    xyz = np.array(xyz, np.float32, order='C', copy=True)
    v = np.array(v, np.float32, order='C', copy=True)
    S, N = xyz.shape[0], xyz.shape[1]
    shared, sptr, sb = _bonds_args(shared_bonds, sbond_ptr, sbonds, S)
    prm = _prm(params, flags)
    rc = c.lib.igm_mstep_md(c.h, 0, ctypes.byref(prm), S, N, xyz.ctypes.data, v.ctypes.data,
                            _np(radii, np.float32).ctypes.data, _np(flags, np.uint32).ctypes.data,
                            shared.ctypes.data if len(shared) else None, len(shared), _lib.ptr(sptr),
                            _lib.ptr(sb), float(evf), float(envf), float(t0), float(t1), float(xmax), int(nsteps))
    c.check(rc, 'igm_mstep_md')
    return xyz, v


def velocity_create(flags, seeds, temperature, ctx=None, device=0):
    """LAMMPS 'velocity nonfixed create T seed' (uniform, loop all, mom yes), one
    velocity set per seed: returns (len(seeds), natom, 3) float32."""
    c = ctx or _lib.context(device)
    flags = _np(flags, np.uint32)
    seeds = _np(seeds, np.int32)
    v = np.zeros((len(seeds), len(flags), 3), np.float32)
    rc = c.lib.igm_velocity_create(c.h, 0, len(seeds), len(flags), flags.ctypes.data, seeds.ctypes.data,
                                   float(temperature), v.ctypes.data)
    c.check(rc, 'igm_velocity_create')
    return v


def act_rows(row, col, dist, prob=None):
    """actdist.hdf5 datasets -> the igm_actdist_row array the GPU consumes."""
    from ._lib import row_dtype
    a = np.zeros(len(row), row_dtype)
    a['row'] = row
    a['col'] = col
    a['dist'] = dist
    if prob is not None:
        a['prob'] = prob
    return a


def hic_select(xyz, radii, chrom, act_row, act_col, act_dist, contact_range=2.0, kspring=1.0,
               inter_class=M.CLASS_INTER_HIC, intra_class=M.CLASS_INTRA_HIC, ctx=None, device=0):
    """Per-structure Hi-C bonds (CSR: ptr (S+1), bonds, class)."""
    c = ctx or _lib.context(device)
    xyz = _np(xyz, np.float32)
    S, N = xyz.shape[0], xyz.shape[1]
    radii = _np(radii, np.float32)
    chrom = _np(chrom, np.int32)
    act = act_rows(act_row, act_col, act_dist)
    ptr = np.zeros(S + 1, np.int64)
    tot = ctypes.c_int64(0)
    args = [c.h, 0, S, N, xyz.ctypes.data, radii.ctypes.data, chrom.ctypes.data, act.ctypes.data,
            len(act), float(contact_range), float(kspring), int(inter_class), int(intra_class), ptr.ctypes.data]
    rc = c.lib.igm_hic_select(*(args + [None, None, ctypes.byref(tot)]))
    c.check(rc, 'igm_hic_select')
    bonds = np.zeros(max(tot.value, 1), bond_dtype)
    cls = np.zeros(max(tot.value, 1), np.int32)
    rc = c.lib.igm_hic_select(*(args + [bonds.ctypes.data, cls.ctypes.data, ctypes.byref(tot)]))
    c.check(rc, 'igm_hic_select')
    return ptr, bonds[:tot.value], cls[:tot.value]


def violations(params, xyz, radii, flags, shared_bonds, shared_class, sbond_ptr, sbonds, sclass, class_cr,
               env_scale, tol, ctx=None, device=0):
    """Per-structure violation records: (S, ncls, 104) int64."""
    c = ctx or _lib.context(device)
    xyz = _np(xyz, np.float32)
    S, N = xyz.shape[0], xyz.shape[1]
    shared, sptr, sb = _bonds_args(shared_bonds, sbond_ptr, sbonds, S)
    shc = _np(shared_class, np.int32) if shared_class is not None else None
    scl = _np(sclass, np.int32) if sclass is not None and sb is not None else None
    ccr = _np(class_cr, np.float64)
    esc = _np(env_scale, np.float64) if env_scale is not None else None
    ncls = len(ccr) + params.nenvelopes
    stats = np.zeros((S, ncls, REC), np.int64)
    prm = _prm(params, flags)
    rc = c.lib.igm_mstep_violations(c.h, 0, ctypes.byref(prm), S, N, xyz.ctypes.data,
                                    _np(radii, np.float32).ctypes.data, _np(flags, np.uint32).ctypes.data,
                                    shared.ctypes.data if len(shared) else None, _lib.ptr(shc), len(shared),
                                    _lib.ptr(sptr), _lib.ptr(sb), _lib.ptr(scl), len(ccr), ccr.ctypes.data,
                                    _lib.ptr(esc), float(tol), stats.ctypes.data)
    c.check(rc, 'igm_mstep_violations')
    return stats
