"""ORACLE (test infrastructure only -- never imported by the product path):
restatement of ExpEnvelope.getScores (igm/model/forces.py:306-417), the violation
score of the volumetric map restraint, pinned against tests/golden/volume_golden.npz
(made by tests/golden/make_golden_volume.py from the reference itself).

Written with the reference's NumPy semantics: the f32 position minus the float64
origin, over the float64 grid; Python round (half to even); -1 outside the grid; the
inside-grid test `id_int.all() >= 0` is always true, so a -1 reads the last voxel
(negative indexing) and the score keeps the -1.  Positions whose rounded index
equals nvoxel raise IndexError in the reference; here they are clamped (the GPU
does the same) -- the goldens exclude them.
"""
import numpy as np


def exp_envelope_scores(pos, vol, k, contact_range=0.95):
    center = np.array(vol['center'], np.float64)
    origin = np.array(vol['origin'], np.float64)
    grid = np.array(vol['grid'], np.float64)
    body = int(vol['body_idx'])
    if body == 0 and k < 0:
        center, origin, grid = center * contact_range, origin * contact_range, grid * contact_range
    if body == 1 and k < 0:
        center, origin, grid = center / contact_range, origin / contact_range, grid / contact_range
    n = np.asarray(vol['nvoxel'])
    mat = vol['matrice']
    out = np.zeros(len(pos))
    for m, p in enumerate(np.asarray(pos, np.float32)):
        idx = (p - origin) / grid
        id_int = np.array([-1 if (idx[d] < 0 or idx[d] >= n[d]) else min(int(round(idx[d])), n[d] - 1)
                           for d in range(3)])
        inside = mat[tuple(id_int) + (3,)]
        if body == 0:
            cond = (inside == 0 and k > 0) or (inside != 0 and k < 0)
        else:
            cond = (inside != 0 and k > 0) or (inside == 0 and k < 0)
        if cond:
            out[m] = _norm(grid * (mat[tuple(id_int)][0:3] - id_int)) / _norm(grid)
    return out


def _norm(v):
    """np.linalg.norm of a float64 3-vector as the reference computed it: sqrt of the
    BLAS ddot, whose two-lane accumulation sums (x0^2 + x2^2) + x1^2 (pinned by the
    goldens; NumPy 2 here would add in index order)."""
    v = [float(t) for t in v]
    return np.sqrt((v[0] * v[0] + v[2] * v[2]) + v[1] * v[1])
