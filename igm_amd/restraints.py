"""M-step restraint assembly for configurations D/E, batched over structures.

Mirrors the per-structure Restraint._apply calls of ModelingStep.task
(igm/steps/ModelingStep.py:399-500):
  * damid_envelope_flags -- Damid._apply_envelope (igm/restraints/damid.py:112-143):
                            the beads of each structure whose shrunk-ellipsoid norm is
                            >= d^2 join a lamina envelope with k = -contact_kspring.
                            Computed on the GPU (igm_damid_select), bit-exact.
  * fish_bonds            -- Fish._apply (igm/restraints/fish.py:85-266): radial
                            (r/R) and pair (p/P) min/max lower/upper bounds to the
                            static centre dummy or between copy pairs, copies ordered
                            by distance (sort_radially / sort_pairs_by_distance, :14-40).
  * sprite_centroids      -- Sprite._apply (igm/restraints/sprite.py:36-71): one
                            mobile centroid per cluster assigned to the structure, at
                            the bead mean, with upper bounds r0 = cbrt(sum r^3 / vf) - r_b.
The structures of a batch share one atom layout: beads, the static centre dummy,
then `nslot` centroid slots; a structure's unused slots are flagged IGM_ATOM_FIXED
(not integrated, no degrees of freedom, no bonds), so every structure sees exactly
the atoms its reference LAMMPS run would have (apart from inert padding).
Bonds come out per structure (lists of igm_bond arrays) for model.concat_bonds.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import bond_dtype, damid_row_dtype, IGM_ATOM_ENV0, IGM_ATOM_FIXED
from .model import LOWER_BOUND_BIT


def _bonds(i, j, r0, k, lower=False):
    b = np.zeros(len(i), bond_dtype)
    b['i'] = i
    b['j'] = np.asarray(j, np.uint32) | (LOWER_BOUND_BIT if lower else np.uint32(0))
    b['r0'] = r0
    b['k'] = k
    return b


def damid_envelope_flags(xyz, radii, rows, semiaxes, contact_range, env_index, base_flags, ctx=None, device=0):
    """Per-structure atom flags (S, N): base_flags | ENV bit of envelope `env_index`
    for the DamID-selected beads of each structure; and rows selected per structure.
    xyz (S, N, 3) f32 struct-major; rows the damid_actdist {loc, dist, prob} rows."""
    c = ctx or _lib.context(device)
    xyz = np.ascontiguousarray(xyz, np.float32)
    S, N = xyz.shape[0], xyz.shape[1]
    radii = np.ascontiguousarray(radii, np.float32)
    base = np.ascontiguousarray(base_flags, np.uint32)
    assert radii.shape == (N,) and base.shape == (N,)
    r = np.zeros(len(rows), damid_row_dtype)
    if len(rows):
        r['loc'], r['dist'], r['prob'] = rows['loc'], rows['dist'], rows['prob']
    abc = np.ascontiguousarray(np.broadcast_to(np.asarray(semiaxes, np.float64), (3,)))
    out = np.zeros((S, N), np.uint32)
    nsel = np.zeros(S, np.int32)
    rc = c.lib.igm_damid_select(c.h, 0, S, N, xyz.ctypes.data, radii.ctypes.data, r.ctypes.data if len(r) else None,
                                len(r), abc.ctypes.data, float(contact_range), int(IGM_ATOM_ENV0 << env_index),
                                base.ctypes.data, out.ctypes.data, nsel.ctypes.data)
    c.check(rc, 'igm_damid_select')
    return out, nsel


def _copies(copy_ptr, copy_idx, h):
    return copy_idx[copy_ptr[h]:copy_ptr[h + 1]]


def fish_bonds(fish, copy_ptr, copy_idx, xyz, struct_ids, rtype, center, tol=10.0, kspring=2.0):
    """Fish._apply for every structure: list of bond arrays (bond order within a
    structure follows the reference's force order).  `fish` is the fish_assignment
    content {'probes', 'radial_min' (nprobe, S_total), 'radial_max', 'pairs',
    'pair_min', 'pair_max'}; struct_ids the global ids of the xyz rows; center the
    index of the static centre dummy."""
    xyz = np.asarray(xyz, np.float32)
    S = xyz.shape[0]
    sid = np.asarray(struct_ids, np.int64)
    ck, tol = float(kspring), float(tol)
    lo = lambda t: np.maximum(0.0, t.astype(np.float64) - tol)  # max(0, target - tol) in float64
    hi = lambda t: t.astype(np.float64) + tol
    parts = []  # (S, k) blocks: i, j, r0, lower -- appended in the reference's order

    def add(i, j, r0, lower):  # every argument is (S, k) or broadcasts to it
        parts.append(tuple(np.broadcast_arrays(np.asarray(i), np.asarray(j), np.asarray(r0, np.float64))) + (lower,))

    cen = np.full((S, 1), center, np.int64)
    if ('r' in rtype or 'R' in rtype) and 'probes' in fish:
        for kind, key in (('r', 'radial_min'), ('R', 'radial_max')):
            if kind not in rtype:
                continue
            for q, h in enumerate(np.asarray(fish['probes'])):
                ii = _copies(copy_ptr, copy_idx, int(h))
                d = np.linalg.norm(xyz[:, ii, :], axis=2)  # (S, nc) float32 norms, as norm(crd[i])
                order = ii[np.argsort(d, axis=1, kind='stable')]  # sort_radially per structure
                t = np.asarray(fish[key])[q][sid][:, None]
                first, last = (order[:, :1], order[:, -1:]) if kind == 'r' else (order[:, -1:], order[:, :1])
                add(cen, first, lo(t), True)
                add(cen, first, hi(t), False)
                if kind == 'r':
                    add(cen, last, hi(t), True)
                else:
                    add(cen, last, t.astype(np.float64) - tol, False)
    if ('p' in rtype or 'P' in rtype) and 'pairs' in fish:
        for kind, key in (('p', 'pair_min'), ('P', 'pair_max')):
            if kind not in rtype:
                continue
            for q, (i, j) in enumerate(np.asarray(fish['pairs'])):
                assert i != j
                ii = _copies(copy_ptr, copy_idx, int(i))
                jj = _copies(copy_ptr, copy_idx, int(j))
                m = np.repeat(ii, len(jj))
                n = np.tile(jj, len(ii))
                d = np.linalg.norm(xyz[:, m, :] - xyz[:, n, :], axis=2)  # (S, ncomb) float32
                o = np.argsort(d, axis=1, kind='stable')  # sort_pairs_by_distance per structure
                sm, sn = m[o], n[o]
                t = np.asarray(fish[key])[q][sid][:, None]
                if kind == 'p':
                    add(sm, sn, np.repeat(lo(t), len(m), axis=1), True)
                    add(sm[:, :1], sn[:, :1], hi(t), False)
                else:
                    add(sm, sn, np.repeat(hi(t), len(m), axis=1), False)
                    add(sm[:, -1:], sn[:, -1:], lo(t), True)
    if not parts:
        return [np.zeros(0, bond_dtype) for _ in range(S)]
    I = np.concatenate([p[0] for p in parts], axis=1)
    J = np.concatenate([p[1] for p in parts], axis=1)
    R = np.concatenate([p[2] for p in parts], axis=1)
    L = np.concatenate([np.full(p[0].shape, p[3]) for p in parts], axis=1)
    out = []
    for s in range(S):
        b = np.zeros(I.shape[1], bond_dtype)
        b['i'] = I[s]
        b['j'] = J[s].astype(np.uint32) | np.where(L[s], LOWER_BOUND_BIT, np.uint32(0)).astype(np.uint32)
        b['r0'] = R[s]
        b['k'] = ck
        out.append(b)
    return out


def cluster_size(radii, volume_occupancy):
    """get_cluster_size (sprite.py:73-79): cbrt(sum r^3 / vf) in float64."""
    return (np.sum(np.asarray(radii, np.float32) ** 3) / volume_occupancy) ** (1. / 3.)


def sprite_centroids(assignment, indptr, selected, xyz, struct_ids, radii, volume_occupancy, kspring, first_slot):
    """Sprite._apply for every structure.  Returns (nslot, pos (S, nslot, 3) f32,
    active (S,) int32, bonds list).  Slot k of structure s is atom first_slot + k."""
    xyz = np.asarray(xyz, np.float32)
    radii = np.asarray(radii, np.float32)
    S = xyz.shape[0]
    assignment = np.asarray(assignment)
    per = [np.where(assignment == int(sid))[0] for sid in struct_ids]
    nslot = max([len(p) for p in per] + [0])
    pos = np.zeros((S, nslot, 3), np.float32)
    active = np.array([len(p) for p in per], np.int32)
    bonds = []
    for s, cids in enumerate(per):
        bl = []
        for k, ci in enumerate(cids):
            beads = np.asarray(selected[indptr[ci]:indptr[ci + 1]], np.int64)
            pos[s, k] = np.mean(xyz[s, beads], axis=0)
            csize = cluster_size(radii[beads], volume_occupancy)
            cen = np.full(len(beads), first_slot + k)
            bl.append(_bonds(beads, cen, np.float64(csize) - radii[beads].astype(np.float64), float(kspring)))
        bonds.append(np.concatenate(bl) if bl else np.zeros(0, bond_dtype))
    return nslot, pos, active, bonds


def centroid_flags(base_flags, active, first_slot, nslot):
    """(S, N) flags: slots >= active[s] are inert (IGM_ATOM_FIXED)."""
    base = np.asarray(base_flags, np.uint32)
    S = len(active)
    f = np.repeat(base[None, :], S, axis=0)
    for s in range(S):
        f[s, first_slot + active[s]:first_slot + nslot] |= np.uint32(IGM_ATOM_FIXED)
    return f
