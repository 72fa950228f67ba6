#!/opt/conda/bin/python3.9
"""Golden vectors for the volumetric map restraint's violation scores, produced by
running the REFERENCE ExpEnvelope.getScores (igm/model/forces.py:306-417) on maps
written in the VolumeFile format and read back by the reference VolumeFile
(igm/utils/files.py:137-166).  Build container only, like make_golden.py:

    /opt/conda/bin/python3.9 tests/golden/make_golden_volume.py

volume_golden.npz: for body 0 (nucleus sphere R=5500, 100 nm grid) and body 1
(nucleolus sphere R=1500 centred off-origin), k = +1 and -1, contact_range 0.95:
the map (nvoxel, center, origin, grid, matrice), 4000 particle positions (f32, some
outside the grid) and the reference's per-particle scores.
"""
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import make_golden  # noqa: E402,F401  (builds the reference environment)
import importlib  # noqa: E402
import numpy as np  # noqa: E402
from igm_amd import volume as V  # noqa: E402  (map construction and .bin writer only)

forces = importlib.import_module('igm.model.forces')
assert np.__version__.startswith('1.')


class P(object):
    def __init__(self, pos):
        self.pos = np.asarray(pos, np.float32)


def main():
    rng = np.random.RandomState(21)
    out = {}
    maps = {0: V.sphere_map(5500.0, 100.0, 3, body_idx=0),
            1: V.sphere_map(1500.0, 100.0, 3, body_idx=1, center=(1000.0, 0.0, 500.0))}
    for body, vol in maps.items():
        span = 7000.0 if body == 0 else 2500.0
        c = np.asarray(vol['center'], np.float64)
        pos = (c + rng.uniform(-span, span, (4600, 3))).astype(np.float32)
        # the reference raises IndexError when round(idx) == nvoxel (idx in [n - 0.5, n));
        # such positions are dropped here (the GPU restatement clamps them)
        n = np.asarray(vol['nvoxel'])
        bad = np.zeros(len(pos), bool)
        for k in (1.0, -1.0):
            o = np.array(vol['origin'], np.float64)
            g = np.array(vol['grid'], np.float64)
            if k < 0:
                o, g = (o * 0.95, g * 0.95) if body == 0 else (o / 0.95, g / 0.95)
            ix = (pos - o) / g
            bad |= np.any((ix >= n - 0.5) & (ix < n), axis=1)
        pos = pos[~bad][:4000]
        parts = [P(x) for x in pos]
        with tempfile.NamedTemporaryFile(suffix='.bin', delete=False) as f:
            name = f.name
        V.write_volume(name, vol)
        for k in (1.0, -1.0):
            f = forces.ExpEnvelope(list(range(len(parts))), volume_file=name, k=k, contact_range=0.95)
            s = f.getScores(parts)
            out['b%d_k%+d_scores' % (body, int(k))] = np.asarray(s, np.float64)
        os.unlink(name)
        for key in ('nvoxel', 'center', 'origin', 'grid', 'matrice'):
            out['b%d_%s' % (body, key)] = vol[key]
        out['b%d_pos' % body] = pos
    np.savez_compressed(os.path.join(HERE, 'volume_golden.npz'), **out)
    print('volume_golden.npz', os.path.getsize(os.path.join(HERE, 'volume_golden.npz')))


if __name__ == '__main__':
    main()
