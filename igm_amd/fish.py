"""FISH A-step (target assignment) on the MI355X.

Mirrors igm/steps/FishAssignmentStep.py task() (py:188-242) for all pairs and probes
at once: per structure the min and max distance over the copies (radial |x| for a
probe, |x_a - x_b| over every copy pair for a pair), the rank of each structure
(argsort(argsort(d)), get_min_max_and_idx py:60-77) and the assigned targets
target[rank].  Returns the fish_restr dictionary of task() with one (index, values)
entry per pair/probe.  No CPU fallback: every value comes from libigmhip.so.
"""
import numpy as np

from . import _lib


def assign(xyz, copy_ptr, copy_idx, kind, items, target_min=None, target_max=None, device=0, ctx=None,
           return_dists=False):
    """kind 'probe' (items: haploid loci) or 'pair' (items: (n, 2) loci).  Targets are
    (nitems, nstruct) sorted distance samples.  Returns (out_min, out_max) -- None
    where the target is absent -- and, with return_dists, the min/max distances."""
    c = ctx or _lib.context(device)
    xyz = np.ascontiguousarray(xyz, np.float32)
    assert xyz.ndim == 3 and xyz.shape[2] == 3, 'xyz must be (nbead, nstruct, 3)'
    copy_ptr = np.ascontiguousarray(copy_ptr, np.int32)
    copy_idx = np.ascontiguousarray(copy_idx, np.int32)
    k = {'probe': 0, 'radial': 0, 'pair': 1}[kind]
    items = np.ascontiguousarray(items, np.int32)
    n = len(items)
    if k == 1:
        assert items.ndim == 2 and items.shape[1] == 2
    nbead, S = xyz.shape[0], xyz.shape[1]
    nhap = len(copy_ptr) - 1

    def tgt(t):
        if t is None:
            return None
        t = np.ascontiguousarray(t, np.float32)
        assert t.shape == (n, S), 'targets must be (nitems, nstruct)'
        return t

    tmin, tmax = tgt(target_min), tgt(target_max)
    omin = np.zeros((n, S), np.float32) if tmin is not None else None
    omax = np.zeros((n, S), np.float32) if tmax is not None else None
    dmin = np.zeros((n, S), np.float32) if return_dists else None
    dmax = np.zeros((n, S), np.float32) if return_dists else None
    rc = c.lib.igm_fish_assign(c.h, 0, xyz.ctypes.data, nbead, S, copy_ptr.ctypes.data, copy_idx.ctypes.data, nhap,
                               k, items.ctypes.data if n else None, n, _lib.ptr(tmin), _lib.ptr(tmax),
                               _lib.ptr(omin), _lib.ptr(omax), _lib.ptr(dmin), _lib.ptr(dmax))
    c.check(rc, 'igm_fish_assign')
    if return_dists:
        return omin, omax, dmin, dmax
    return omin, omax


def task(xyz, copy_ptr, copy_idx, fish_input, device=0, ctx=None):
    """fish_restr of FishAssignmentStep.task for the whole input (every batch):
    fish_input is the dict view of the FISH h5 ('pairs', 'probes', 'pair_min', ...).
    Returns {'pair_min': [(index, assigned)], 'radial_min': [...], ...}."""
    out = {'pair_min': [], 'radial_min': [], 'pair_max': [], 'radial_max': []}
    for kind, key, pre in (('pair', 'pairs', 'pair'), ('probe', 'probes', 'radial')):
        if key not in fish_input:
            continue
        items = np.asarray(fish_input[key])
        if kind == 'pair':  # the first row equal to the pair (py:211)
            _, idx, inv = np.unique(items, axis=0, return_index=True, return_inverse=True)
            first = idx[np.ravel(inv)]
        else:  # exactly one row equal to the probe, else ValueError (py:226-229)
            first = np.arange(len(items))
            u, cnt = np.unique(items, return_counts=True)
            if np.any(cnt != 1):
                raise ValueError(f"Cannot find probe: {u[cnt != 1][0]}")
        tmin, tmax = fish_input.get(pre + '_min'), fish_input.get(pre + '_max')
        omin, omax = assign(xyz, copy_ptr, copy_idx, kind, items,
                            None if tmin is None else np.asarray(tmin)[first],
                            None if tmax is None else np.asarray(tmax)[first], device=device, ctx=ctx)
        for q in range(len(items)):
            if omin is not None:
                out[pre + '_min'].append((int(first[q]), omin[q]))
            if omax is not None:
                out[pre + '_max'].append((int(first[q]), omax[q]))
    return out
